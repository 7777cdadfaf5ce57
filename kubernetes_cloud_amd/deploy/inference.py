"""KServe InferenceServices, download / serialize / convert Jobs (S1-S15, D1).

One manifest set per reference online-inference example, rewritten for MI355X
nodes and this framework's entrypoints:

* stable-diffusion (S3): PVC, model download Job, optional tensorize Job, ISVC
  running ``serving.sd_service`` (micro-batched, ``containerConcurrency`` 8
  instead of 1 because requests are batched on the GPU).
* bloom-176b (S4/S5): PVC, download Job, ISVC running ``serving.tp_server``
  under torchrun over the 8 GPUs of one node (TP=8 over xGMI) -- replaces both
  the 5-GPU accelerate layer split and the DeepSpeed-Inference image.
* fastertransformer (S6): model-store convert Jobs (GPT-J, GPT-NeoX) and
  Triton-protocol ISVCs (``serving.triton_ft``, model name fastertransformer,
  port 80) -- the FT client talks to it unchanged.
* tensorizer-isvc (S8): download+serialize Job (``gptj.tensors``), KServe ISVCs
  for ``MODEL_LOAD_TYPE=tensorizer|hf`` and the plain-text (Flask-API) variant.
* gpt-2 (S10) predictor + transformer, aitextgen (S15), custom predictor
  pattern (S14).
"""
from __future__ import annotations

from .k8s import GPU_CLASS_LABEL, ROCM_ENV, affinity, image, pvc, resources

MI355X = "MI355X"


def _isvc(name: str, containers: list, annotations: dict | None = None, min_replicas: int = 0,
          max_replicas: int = 1, concurrency: int | None = None, transformer: dict | None = None,
          gpu_class: str = MI355X, region: str | None = None) -> dict:
    pred = {"minReplicas": min_replicas, "maxReplicas": max_replicas, "affinity": affinity(gpu_class, region),
            "containers": containers}
    if concurrency:
        pred["containerConcurrency"] = concurrency
    spec = {"predictor": pred}
    if transformer:
        spec["transformer"] = transformer
    md = {"name": name}
    if annotations:
        md["annotations"] = annotations
    return {"apiVersion": "serving.kserve.io/v1beta1", "kind": "InferenceService", "metadata": md, "spec": spec}


def _container(command, args=None, env=None, gpus=1, cpu=8, memory="64Gi", port=None, probe_path=None):
    c = {"name": "kserve-container", "image": image(), "imagePullPolicy": "IfNotPresent", "command": command,
         "env": list(env or []) + list(ROCM_ENV), "resources": resources(gpus=gpus, cpu=cpu, memory=memory)}
    if args:
        c["args"] = args
    if port:
        c["ports"] = [{"containerPort": port, "protocol": "TCP"}]
    if probe_path:
        c["readinessProbe"] = {"httpGet": {"path": probe_path, "port": port or 8080}, "initialDelaySeconds": 30,
                               "periodSeconds": 10}
    return c


def _job(name: str, command, args, claim: str, mount: str = "/mnt/models", gpus=None, cpu=8, memory="64Gi",
         env=None, gpu_class=None) -> dict:
    c = {"name": name, "image": image(), "command": command, "args": args,
         "env": list(env or []) + list(ROCM_ENV),
         "resources": resources(gpus=gpus, cpu=cpu, memory=memory),
         "volumeMounts": [{"name": "model-storage", "mountPath": mount}]}
    spec = {"containers": [c], "restartPolicy": "Never",
            "volumes": [{"name": "model-storage", "persistentVolumeClaim": {"claimName": claim}}]}
    if gpu_class:
        spec["affinity"] = affinity(gpu_class, None)
    return {"apiVersion": "batch/v1", "kind": "Job", "metadata": {"name": name},
            "spec": {"backoffLimit": 2, "template": {"spec": spec}}}


HF_TOKEN_ENV = [{"name": "HUGGING_FACE_HUB_TOKEN", "valueFrom": {"secretKeyRef": {
    "name": "huggingface-hub-token", "key": "token", "optional": True}}}]


def stable_diffusion() -> dict:
    model = "runwayml/stable-diffusion-v1-5"
    s3 = lambda n, k: {"apiVersion": "v1", "kind": "Secret", "type": "Opaque", "metadata": {"name": n},  # noqa: E731
                       "data": {k: "<base64-encoded-value>"}}
    upload = _job("stable-diffusion-uploader", ["python3", "-m", "kubernetes_cloud_amd.io.s3_upload"],
                  ["--src", f"/mnt/models/{model}", "--dest", "s3://<BUCKET>/", "--acl-public"],
                  "stable-diffusion-models", cpu=1, memory="2Gi",
                  env=[{"name": "AWS_KEY", "valueFrom": {"secretKeyRef": {"name": "s3-access-key", "key": "access_key"}}},
                       {"name": "AWS_SECRET", "valueFrom": {"secretKeyRef": {"name": "s3-secret-key",
                                                                              "key": "secret_key"}}},
                       {"name": "AWS_HOST", "valueFrom": {"secretKeyRef": {"name": "s3-host-url", "key": "url"}}}])
    return {
        "01-optional-s3-secret.yaml": [s3("s3-access-key", "access_key"), s3("s3-secret-key", "secret_key"),
                                       s3("s3-host-url", "url")],
        "03-optional-s3-upload-job.yaml": upload,
        "00-model-pvc.yaml": pvc("stable-diffusion-models", "100Gi"),
        "02-model-download-job.yaml": _job(
            "stable-diffusion-download", ["python3", "-m", "kubernetes_cloud_amd.data.downloader"],
            ["-model", model, "-dest", f"/mnt/models/{model}", "-type", "diffusers"], "stable-diffusion-models",
            env=HF_TOKEN_ENV, cpu=4, memory="16Gi"),
        "02-optional-serialize-job.yaml": _job(
            "stable-diffusion-serialize", ["python3", "-c",
                                           "from kubernetes_cloud_amd.serving.sd_service import serialize_main; "
                                           "serialize_main()"],
            ["--model-id", f"/mnt/models/{model}", "--save-path", f"/mnt/models/{model}-tensorized"],
            "stable-diffusion-models", cpu=8, memory="32Gi"),
        "03-inference-service.yaml": _isvc(
            "stable-diffusion", [_container(
                ["python3", "-m", "kubernetes_cloud_amd.serving.sd_service"],
                ["--model-id", f"/mnt/pvc/{model}"],
                env=[{"name": "STORAGE_URI", "value": "pvc://stable-diffusion-models/"},
                     {"name": "NUM_INFERENCE_STEPS", "value": "50"}, {"name": "CONDITION_SCALE", "value": "7.0"},
                     {"name": "MAX_BATCH", "value": "8"}], cpu=8, memory="48Gi")],
            annotations={"autoscaling.knative.dev/scaleToZeroPodRetentionPeriod": "20m"}, concurrency=8),
    }


def bloom_176b() -> dict:
    env = [{"name": "MODEL_ID", "value": "bigscience/bloom"}, {"name": "MODEL_PATH", "value": "/mnt/pvc/bloom"},
           {"name": "MODEL_DOWNLOAD_TIMEOUT", "value": "3600"}, {"name": "MIN_LENGTH", "value": "1"},
           {"name": "MAX_LENGTH", "value": "40"}, {"name": "TEMPERATURE", "value": "1.0"},
           {"name": "TOP_K", "value": "50"}, {"name": "TOP_P", "value": "1.0"},
           {"name": "REPETITION_PENALTY", "value": "1.0"},
           {"name": "STORAGE_URI", "value": "pvc://bloom-176b-models/"}]
    c = _container(["torchrun", "--standalone", "--nproc-per-node", "8", "-m",
                    "kubernetes_cloud_amd.serving.tp_server"], ["--model-path", "/mnt/pvc/bloom", "--port", "8080"],
                   env=env, gpus=8, cpu=96, memory="512Gi", port=8080, probe_path="/v1/models/bigscience-bloom")
    c["volumeMounts"] = [{"name": "dshm", "mountPath": "/dev/shm"}]
    isvc = _isvc("bloom-176b", [c], annotations={"autoscaling.knative.dev/scaleToZeroPodRetentionPeriod": "60m"})
    isvc["spec"]["predictor"]["volumes"] = [{"name": "dshm", "emptyDir": {"medium": "Memory"}}]
    return {
        "00-bloom-176b-pvc.yaml": pvc("bloom-176b-models", "400Gi"),
        "01-bloom-176b-download-job.yaml": _job(
            "bloom-176b-download", ["python3", "-m", "kubernetes_cloud_amd.data.downloader"],
            ["-model", "bigscience/bloom", "-dest", "/mnt/pvc/bloom", "-ready"], "bloom-176b-models",
            mount="/mnt/pvc", env=HF_TOKEN_ENV, cpu=16, memory="32Gi"),
        "02-bloom-176b-inferenceservice.yaml": isvc,
    }


def bloom_176b_deepspeed() -> dict:
    """online-inference/bloom-176b-deepspeed (S5): the pre-sharded
    microsoft/bloom-deepspeed-inference-fp16 checkpoint downloaded into the HF
    hub cache on a PVC (01-download-job.yaml: download.py --model-id --revision,
    HF_HOME=/mnt/models), served TP=8 on one MI355X node on port 5000 with the
    bloom-inference-server routes (02-inference-service.yaml:22-45)."""
    repo = "microsoft/bloom-deepspeed-inference-fp16"
    name = "microsoft-bloom-deepspeed-inference-fp16"
    dl = _job(f"{name}-download", ["python3", "-m", "kubernetes_cloud_amd.data.hf_snapshot"],
              [f"--model-id={repo}", "--revision=main"], name, mount="/mnt/models",
              env=[{"name": "HF_HOME", "value": "/mnt/models"}] + HF_TOKEN_ENV, cpu=4, memory="16Gi")
    c = _container(["torchrun", "--standalone", "--nproc-per-node", "8", "-m",
                    "kubernetes_cloud_amd.serving.tp_server"], ["--model-name", repo, "--port", "5000"],
                   env=[{"name": "STORAGE_URI", "value": f"pvc://{name}/"}, {"name": "HF_HOME", "value": "/mnt/models"},
                        {"name": "MODEL_NAME", "value": repo}],
                   gpus=8, cpu=96, memory="512Gi", port=5000)
    c["volumeMounts"] = [{"name": "dshm", "mountPath": "/dev/shm"}]
    isvc = _isvc(name, [c], min_replicas=1, concurrency=1)
    isvc["spec"]["predictor"]["volumes"] = [{"name": "dshm", "emptyDir": {"medium": "Memory"}}]
    return {"00-pvc.yaml": pvc(name, "400Gi"), "01-download-job.yaml": dl, "02-inference-service.yaml": isvc}


def fastertransformer() -> dict:
    out = {"model-storage-pvc.yml": pvc("ft-model-storage", "200Gi")}
    for name, model, store in (("gptj", "EleutherAI/gpt-j-6B", "gptj-store"),
                               ("neox", "EleutherAI/gpt-neox-20b", "neox-store")):
        out[f"download-weights-job-{name}.yml"] = _job(
            f"ft-{name}-download-convert", ["bash", "-c"],
            [f"python3 -m kubernetes_cloud_amd.data.downloader -model {model} -dest /mnt/pvc/{name}-hf && "
             f"python3 -c 'from kubernetes_cloud_amd.serving.triton_ft import convert_main; convert_main()' "
             f"--model-dir /mnt/pvc/{name}-hf --output-dir /mnt/pvc/{store}/triton-model-store "
             f"--n-inference-gpus 1 --data-type fp16"],
            "ft-model-storage", mount="/mnt/pvc", env=HF_TOKEN_ENV, cpu=16, memory="128Gi")
        c = _container(["python3", "-m", "kubernetes_cloud_amd.serving.triton_ft"],
                       ["--model-store", f"/mnt/pvc/{store}/triton-model-store", "--http-port", "80"],
                       env=[{"name": "STORAGE_URI", "value": "pvc://ft-model-storage/"},
                            {"name": "MAX_BATCH", "value": "64"}], cpu=16, memory="96Gi", port=80,
                       probe_path="/v2/health/ready")
        out[f"ft-inference-service-{name}.yml"] = _isvc(f"fastertransformer-{name}", [c])
    return out


def tensorizer_isvc() -> dict:
    dl = _job("gptj-model-download", ["bash", "-c"],
              ["python3 -m kubernetes_cloud_amd.data.downloader -model EleutherAI/gpt-j-6B -dest /mnt/pvc "
               "-tensorize gptj.tensors -dtype float16"], "model-storage", mount="/mnt/pvc", env=HF_TOKEN_ENV,
              cpu=8, memory="64Gi")
    out = {"pvc.yaml": pvc("model-storage", "50Gi"), "model-download/model-download-job.yaml": dl}
    for kind, load in (("tensorizer", "tensorizer"), ("hf", "hf")):
        env = [{"name": "MODEL_LOAD_TYPE", "value": load}, {"name": "STORAGE_URI", "value": "pvc://model-storage/"},
               {"name": "MODEL_PATH", "value": "/mnt/pvc"}]
        out[f"kserve/{kind}-isvc.yaml"] = _isvc(
            f"gptj-{kind}", [_container(["python3", "-c",
                                         "from kubernetes_cloud_amd.serving.predictors import gptj_main; gptj_main()"],
                                        env=env, cpu=8, memory="48Gi")],
            annotations={"autoscaling.knative.dev/target": "1"}, max_replicas=100)
        out[f"flask/{kind}-isvc.yaml"] = _isvc(
            f"gptj-{kind}-text", [_container(["python3", "-c", "from kubernetes_cloud_amd.serving.predictors "
                                                              "import gptj_text_main; gptj_text_main()"],
                                             env=env + [{"name": "PORT", "value": "8000"}], cpu=8, memory="48Gi",
                                             port=8000, probe_path="/")], max_replicas=100)
    return out


def gpt2() -> dict:
    """online-inference/gpt-2: PVC-backed ISVC (124M and the 1558M "huge" model,
    service-pvc/*.yaml) and the S3-backed one with its credentials secret and
    service account (service-s3/*.yaml: KServe's storage initializer pulls
    storageUri with the SA's secret; target concurrency 4), each predictor +
    BPE transformer."""
    def pair(name, model_path, storage_uri, sa=None, concurrency=4, max_replicas=2, transformer_par=None):
        pred = _container(["python3", "-c", "from kubernetes_cloud_amd.serving.predictors import "
                                            "gpt2_predictor_main; gpt2_predictor_main()"],
                          env=[{"name": "MODEL_PATH", "value": model_path},
                               {"name": "STORAGE_URI", "value": storage_uri}], cpu=4, memory="16Gi")
        tr = {"containers": [{"name": "kserve-container", "image": image(),
                              "command": ["python3", "-c", "from kubernetes_cloud_amd.serving.predictors import "
                                                           "gpt2_transformer_main; gpt2_transformer_main()"],
                              "args": ["--model_name", name], "env": [{"name": "TOKENIZER_PATH",
                                                                       "value": model_path}]}],
              "minReplicas": 0, "maxReplicas": transformer_par or 1}
        isvc = _isvc(name, [pred], transformer=tr, concurrency=concurrency, max_replicas=max_replicas,
                     annotations={"autoscaling.knative.dev/target": str(concurrency)})
        if sa:
            isvc["spec"]["predictor"]["serviceAccountName"] = sa
        return isvc
    s3_secret = {"apiVersion": "v1", "kind": "Secret", "type": "Opaque",
                 "metadata": {"name": "s3-secret", "annotations": {"serving.kserve.io/s3-endpoint": "object.ord1.coreweave.com",
                                                                   "serving.kserve.io/s3-usehttps": "1"}},
                 "data": {"AWS_ACCESS_KEY_ID": "<base64-encoded-value>",
                          "AWS_SECRET_ACCESS_KEY": "<base64-encoded-value>"}}
    sa = {"apiVersion": "v1", "kind": "ServiceAccount", "metadata": {"name": "s3-sa"},
          "secrets": [{"name": "s3-secret"}]}
    return {
        "gpt-pvc-inferenceservice.yaml": pair("gpt-2", "/mnt/pvc/gpt2", "pvc://model-storage/"),
        "service-pvc/gpt-pvc-huge-model-inferenceservice.yaml": pair(
            "gpt-pvc-huge", "/mnt/models", "pvc://model-storage/1558M/", max_replicas=20, transformer_par=2),
        "service-s3/s3-secret.yaml": s3_secret,
        "service-s3/s3-serviceaccount.yaml": sa,
        "service-s3/gpt-s3-inferenceservice.yaml": pair("gpt-s3", "/mnt/models", "s3://coreweave/gpt-2/124M/",
                                                        sa="s3-sa"),
    }


def image_classifier() -> dict:
    """online-inference/image-classifier (S11): classifier ISVC + b64/url transformer
    (service/classifier-inferenceservice.yaml:1-47), PyTorch model on the PVC."""
    pred = _container(["python3", "-c", "from kubernetes_cloud_amd.serving.predictors import "
                                        "image_classifier_main; image_classifier_main()"],
                      env=[{"name": "MODEL_PATH", "value": "/mnt/models/resnet50_imagenet.pt"},
                           {"name": "MODEL_NAME", "value": "image-classifier"},
                           {"name": "STORAGE_URI", "value": "pvc://model-storage/classifier/"}], cpu=4, memory="8Gi")
    return {"service/classifier-inferenceservice.yaml": _isvc("image-classifier", [pred], max_replicas=4,
                                                              concurrency=8),
            "model-storage-pvc.yaml": pvc("model-storage", "20Gi")}


def custom_sentiment() -> dict:
    """online-inference/custom-sentiment (S14): PVC-loaded custom predictor
    (sentiment-inferenceservice.yaml), a sleep Deployment that mounts the PVC
    for copying the model in (sleep-deployment.yaml), and the image-pull
    secret patch of the default service account."""
    c = _container(["python3", "/app/model.py"], env=[{"name": "STORAGE_URI", "value": "pvc://model-storage/sentiment"}],
                   cpu=3, memory="8Gi")
    isvc = _isvc("sentiment", [c], max_replicas=10, concurrency=1)
    isvc["metadata"]["labels"] = {"qos.coreweave.cloud/latency": "low"}
    sleep = {"apiVersion": "apps/v1", "kind": "Deployment", "metadata": {"name": "sleep"},
             "spec": {"replicas": 1, "revisionHistoryLimit": 1, "strategy": {"type": "Recreate"},
                      "selector": {"matchLabels": {"app.kubernetes.io/name": "sleep"}},
                      "template": {"metadata": {"labels": {"app.kubernetes.io/name": "sleep"}},
                                   "spec": {"containers": [{
                                       "name": "sleep", "image": image(), "command": ["sleep"], "args": ["86400d"],
                                       "imagePullPolicy": "IfNotPresent",
                                       "resources": {"requests": {"cpu": "50m", "memory": "10Mi"},
                                                     "limits": {"cpu": 1, "memory": "128Mi"}},
                                       "volumeMounts": [{"name": "model-storage", "mountPath": "/models"}]}],
                                       "volumes": [{"name": "model-storage",
                                                    "persistentVolumeClaim": {"claimName": "model-storage"}}]}}}}
    patch = {"apiVersion": "v1", "kind": "ServiceAccount", "imagePullSecrets": [{"name": "docker-hub"}]}
    return {"sentiment-inferenceservice.yaml": isvc, "sleep-deployment.yaml": sleep,
            "model-storage-pvc.yaml": pvc("model-storage", "20Gi"),
            "image-secrets-serviceaccount.patch.yaml": patch}


def aitextgen() -> dict:
    return {"aitextgen-inferenceservice.yaml": _isvc(
        "aitextgen", [_container(["python3", "-c", "from kubernetes_cloud_amd.serving.predictors import "
                                                   "aitextgen_main; aitextgen_main()"],
                                 env=[{"name": "MODEL_PATH", "value": "/mnt/pvc/gpt2-xl"},
                                      {"name": "STORAGE_URI", "value": "pvc://model-storage/"}],
                                 cpu=4, memory="32Gi")])}


def dalle_mini() -> dict:
    """online-inference/dalle-mini: PVC, downloader job (.ready.txt), InferenceService with the
    generation defaults as env (02-inference-service.yaml:33-47); PyTorch-ROCm predictor."""
    model = "dalle-mini/dalle-mega"
    env = [{"name": "MODEL_ID", "value": model}, {"name": "MODEL_CACHE", "value": "/mnt/models"},
           {"name": "STORAGE_URI", "value": "pvc://dalle-mini-model-cache/"},
           {"name": "TOP_K", "value": "50"}, {"name": "TOP_P", "value": "1.0"},
           {"name": "TEMPERATURE", "value": "1.0"}, {"name": "CONDITION_SCALE", "value": "10.0"}]
    return {
        "00-model-pvc.yaml": pvc("dalle-mini-model-cache", "100Gi"),
        "01-model-download-job.yaml": _job(
            "dalle-mini-download", ["python3", "-m", "kubernetes_cloud_amd.data.downloader"],
            ["-model", model, "-dest", f"/mnt/models/{model}"], "dalle-mini-model-cache", cpu=4, memory="16Gi"),
        "02-inference-service.yaml": _isvc(
            "dalle-mega", [_container(["python3", "-m", "kubernetes_cloud_amd.serving.dalle_service"], env=env,
                                      cpu=6, memory="48Gi")], min_replicas=1, concurrency=1),
    }


def custom_predictor() -> dict:
    """S13/S14 pattern: bring-your-own predictor subclassing serving.server.Model."""
    return {"custom-inferenceservice.yaml": _isvc(
        "custom-model", [_container(["python3", "/app/model.py"], gpus=1, cpu=4, memory="16Gi")]),
        "model-storage-pvc.yaml": pvc("model-storage", "20Gi")}


__all__ = ["stable_diffusion", "bloom_176b", "bloom_176b_deepspeed", "fastertransformer", "tensorizer_isvc", "gpt2",
           "image_classifier", "custom_sentiment", "aitextgen", "custom_predictor", "GPU_CLASS_LABEL"]
