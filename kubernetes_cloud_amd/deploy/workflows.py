"""Argo workflows / templates / event bindings for MI355X (T7, T10, T11, T12, P1).

Same parameter surfaces as the reference workflows (SURVEY §2.6 item 13:
finetune-workflow.yaml:8-199, sd-finetune-workflow-template.yaml:9-118,
db-workflow-template.yaml:9-105, gpt-neox 04-finetune-workflow.yaml:8-85, event
payload mappings sd-finetune-workflow-event-binding.yaml:11-24 and
db-workflow-event-binding.yaml:11-39), so existing ``argo submit -p ...`` calls
and event payloads keep working. What changes: every GPU step runs the one
ROCm/gfx950 image of this framework (``python -m kubernetes_cloud_amd...``
entrypoints), requests ``amd.com/gpu`` on MI355X-labelled nodes, multi-GPU
steps launch one process per GPU with ``kubernetes_cloud_amd.launch`` /
torchrun over RCCL, and the GPU/RAM defaults are sized for 288 GB HBM nodes.
"""
from __future__ import annotations

from .k8s import ROCM_ENV, affinity, image, ip, pvc_volume, resources, shm_volume, wp

MI355X = "MI355X"


def _params(pairs):
    out = []
    for k, v in pairs:
        out.append({"name": k} if v is None else {"name": k, "value": v})
    return out


def _args(names):
    return {"parameters": [{"name": n, "value": wp(n)} for n in names]}


def _vol_mount(pvc_param="pvc"):
    return {"mountPath": "/" + wp(pvc_param), "name": wp(pvc_param)}


# ------------------------------------------------------------------ T7
FINETUNE_PARAMS = [
    ("run_name", None), ("pvc", "finetune-data"), ("model", "EleutherAI/pythia-2.8b-deduped"),
    ("dataset", "dataset"), ("trust_remote_code", "false"), ("tensorizer_uri", ""), ("retokenize", "true"),
    ("sanitize", "true"), ("tokenizer", ""), ("reorder", ""), ("no_shuffle", "false"), ("sampling", "100"),
    ("eot_token", ""), ("pad_token", ""), ("boundary_token", "\\n"), ("boundary_index", "-1"),
    ("context", "2048"), ("prompt_file", ""), ("prompt_every", "0"), ("prompt_tokens", "200"),
    ("prompt_samples", "5"), ("top_k", "50"), ("top_p", "0.95"), ("temperature", "1.0"),
    ("repetition_penalty", "1.1"), ("warmup_ratio", "0.1"), ("batch_size", "-1"), ("force_fp16", "false"),
    ("batch_size_divisor", "1.0"), ("random_seed", "42"), ("learn_rate", "5e-5"), ("epochs", "1"),
    ("gradients", "5"), ("zero_stage", "1"), ("save_steps", "500"), ("no_resume", "false"), ("logs", "logs"),
    ("wandb_key", ""), ("project_id", "huggingface"), ("run_inference", "false"), ("inference_only", "false"),
    ("download_dataset", "false"), ("region", "ORD1"), ("trainer_gpu", MI355X), ("trainer_gpus", 1),
    ("trainer_cores", 16), ("trainer_ram", 256), ("inference_gpu", MI355X),
    ("model_downloader_image", "ghcr.io/kubernetes-cloud-amd/kca"), ("model_downloader_tag", "rocm7.2-gfx950"),
    ("tokenizer_image", "ghcr.io/kubernetes-cloud-amd/kca"), ("tokenizer_tag", "rocm7.2-gfx950"),
    ("dataset_downloader_image", "ghcr.io/coreweave/dataset-downloader/smashwords-downloader"),
    ("dataset_downloader_tag", "cd6408a"), ("finetuner_image", "ghcr.io/kubernetes-cloud-amd/kca"),
    ("finetuner_tag", "rocm7.2-gfx950"),
]

_TOKENS = ("/{{workflow.parameters.pvc}}/{{workflow.parameters.dataset}}-"
           "{{=sprig.replace('/', '_', sprig.replace('.','_', sprig.replace('-','_', workflow.parameters.model)))}}"
           "-{{workflow.parameters.context}}-b{{workflow.parameters.boundary_index}}"
           "-{{workflow.parameters.tokenizer_tag}}.tokens")


def _cpu_step(name, inputs, img, command, args, cpu="4", mem="2Gi", region=True):
    t = {"name": name, "retryStrategy": {"limit": 1},
         "container": {"image": img, "command": command, "args": args, "env": list(ROCM_ENV),
                       "resources": resources(cpu=cpu, memory=mem), "volumeMounts": [_vol_mount()]},
         "volumes": [pvc_volume(wp("pvc"))], "affinity": affinity(None, wp("region") if region else None)}
    if inputs:
        t["inputs"] = {"parameters": [{"name": n} for n in inputs]}
    return t


def finetune_workflow() -> dict:
    finetuner_flags = " ".join([
        "--run-name={{workflow.parameters.run_name}}",
        "--model=/{{workflow.parameters.pvc}}/models/{{workflow.parameters.model}}",
        "--trust-remote-code={{workflow.parameters.trust_remote_code}}",
        "--dataset " + _TOKENS,
        "--tensorizer-uri='{{workflow.parameters.tensorizer_uri}}'",
        "--lr={{workflow.parameters.learn_rate}}", "--epochs={{workflow.parameters.epochs}}",
        "--train-ratio=1.0", "--eot='{{workflow.parameters.eot_token}}'",
        "--pad='{{workflow.parameters.pad_token}}'", "--warmup-ratio={{workflow.parameters.warmup_ratio}}",
        "--bs={{workflow.parameters.batch_size}}", "--bs-divisor={{workflow.parameters.batch_size_divisor}}",
        "--gradients={{workflow.parameters.gradients}}", "--zero-stage={{workflow.parameters.zero_stage}}",
        "--seed={{workflow.parameters.random_seed}}", "--output-path=/{{workflow.parameters.pvc}}/finetunes/",
        "--no-resume={{workflow.parameters.no_resume}}", "--cache=/{{workflow.parameters.pvc}}/cache/",
        "--save-steps={{workflow.parameters.save_steps}}", "--context-size={{workflow.parameters.context}}",
        "--project-id={{workflow.parameters.project_id}}",
        "--logs=/{{workflow.parameters.pvc}}/{{workflow.parameters.logs}}",
        "--fp16={{workflow.parameters.force_fp16}}", "--no-shuffle={{workflow.parameters.no_shuffle}}",
        "--prompt-file={{=workflow.parameters.prompt_file == '' ? '' : '/' + workflow.parameters.pvc + '/' + "
        "workflow.parameters.prompt_file}}",
        "--prompt-every={{workflow.parameters.prompt_every}}", "--prompt-tokens={{workflow.parameters.prompt_tokens}}",
        "--prompt-samples={{workflow.parameters.prompt_samples}}", "--top-k={{workflow.parameters.top_k}}",
        "--top-p={{workflow.parameters.top_p}}", "--temperature={{workflow.parameters.temperature}}",
        "--repetition-penalty={{workflow.parameters.repetition_penalty}}",
    ])
    main = {"name": "main", "steps": [
        [{"name": "check-model", "template": "check-model", "arguments": _args(["model"]),
          "when": "'{{workflow.parameters.tensorizer_uri}}' == ''"}],
        # weights come from the PVC unless they stream from a tensorized URI (the finetuner's
        # --tensorizer-uri, or its probe of the public bucket when check-model found the model);
        # config + tokenizer always land on the PVC (the finetuner and the tokenizer step read them)
        [{"name": "model-downloader", "template": "model-downloader",
          "arguments": {"parameters": [{"name": "model", "value": wp("model")},
                                       {"name": "dest", "value": "/" + wp("pvc") + "/models/" + wp("model")},
                                       {"name": "tokenizer_only", "value": "{{steps.check-model.outputs.result}}"}]},
          "when": "'{{workflow.parameters.tensorizer_uri}}' == ''"},
         {"name": "model-downloader-tokenizer", "template": "model-downloader",
          "arguments": {"parameters": [{"name": "model", "value": wp("model")},
                                       {"name": "dest", "value": "/" + wp("pvc") + "/models/" + wp("model")},
                                       {"name": "tokenizer_only", "value": "true"}]},
          "when": "'{{workflow.parameters.tensorizer_uri}}' != ''"}],
        [{"name": "dataset-downloader", "template": "dataset-downloader",
          "arguments": {"parameters": [{"name": "output", "value": "/" + wp("pvc") + "/" + wp("dataset")}]},
          "when": "{{workflow.parameters.inference_only}} == false && {{workflow.parameters.download_dataset}} == true"}],
        [{"name": "tokenizer", "template": "model-tokenizer", "when": "{{workflow.parameters.inference_only}} == false",
          "arguments": {"parameters": [
              {"name": "input", "value": "/" + wp("pvc") + "/" + wp("dataset")},
              {"name": "output", "value": _TOKENS},
              {"name": "tokenizer", "value": "{{=sprig.default('/' + workflow.parameters.pvc + '/models/' + "
                                             "workflow.parameters.model, workflow.parameters.tokenizer)}}"},
              {"name": "context", "value": wp("context")}, {"name": "eot", "value": wp("eot_token")},
              {"name": "pad", "value": wp("pad_token")}, {"name": "boundary", "value": wp("boundary_token")},
              {"name": "boundary_index", "value": wp("boundary_index")}, {"name": "reorder", "value": wp("reorder")},
              {"name": "sampling", "value": wp("sampling")}, {"name": "sanitize", "value": wp("sanitize")},
              {"name": "retokenize", "value": wp("retokenize")}]}}],
        [{"name": "finetuner", "template": "model-finetuner", "when": "{{workflow.parameters.inference_only}} == false",
          "arguments": {"parameters": [{"name": "finetuner_params", "value": finetuner_flags},
                                       {"name": "wandb_key", "value": wp("wandb_key")}]}}],
        [{"name": "inference-service", "template": "model-inference-service",
          "when": "{{workflow.parameters.run_inference}} == true",
          "arguments": {"parameters": [
              {"name": "model_path", "value": "finetunes/results-{{workflow.parameters.run_name}}/final"},
              {"name": "model_name", "value": "final"}]}}],
    ]}
    kca = image("finetuner_tag", "finetuner_image")
    check = {"name": "check-model", "inputs": {"parameters": [{"name": "model"}]}, "retryStrategy": {"limit": 1},
             "container": {"image": kca, "command": ["python3", "-m", "kubernetes_cloud_amd.data.downloader"],
                           "args": ["check-tensorized", "-model", ip("model"), "-out", "/tmp/output.txt"]},
             "outputs": {"parameters": [{"name": "result", "valueFrom": {"path": "/tmp/output.txt"}}]}}
    dl = _cpu_step("model-downloader", ["model", "dest", "tokenizer_only"],
                   image("model_downloader_tag", "model_downloader_image"),
                   ["python3", "-m", "kubernetes_cloud_amd.data.downloader"],
                   ["-model", ip("model"), "-dest", ip("dest"), "-tokenizer-only", ip("tokenizer_only")],
                   cpu="4", mem="8Gi")
    dsd = _cpu_step("dataset-downloader", ["output"], image("dataset_downloader_tag", "dataset_downloader_image"),
                    ["/ko-app/smashwords-downloader"], ["--data_dir", ip("output")], cpu="4", mem="1Gi")
    tok = _cpu_step("model-tokenizer", ["input", "tokenizer", "context", "eot", "pad", "output", "boundary",
                                        "boundary_index", "sampling", "reorder", "sanitize", "retokenize"],
                    image("tokenizer_tag", "tokenizer_image"), ["python3", "-m", "kubernetes_cloud_amd.data.tokenizer"],
                    ["-tokenizer", ip("tokenizer"), "-context", ip("context"), "-eot", ip("eot"), "-pad", ip("pad"),
                     "-input", ip("input"), "-output", ip("output"), "-boundary", ip("boundary"),
                     "-boundary_overlap", ip("boundary_index"), "-reorder", ip("reorder"),
                     "-sampling", ip("sampling"), "-sanitize=" + ip("sanitize"), "-retokenize=" + ip("retokenize")],
                    cpu="16", mem="16Gi")
    ft = {
        "name": "model-finetuner",
        "inputs": {"parameters": [{"name": "finetuner_params"}, {"name": "wandb_key"}]},
        "podSpecPatch": ("containers:\n  - name: main\n    resources:\n"
                         "      requests: {memory: \"{{workflow.parameters.trainer_ram}}Gi\", "
                         "cpu: \"{{workflow.parameters.trainer_cores}}\", "
                         "amd.com/gpu: \"{{workflow.parameters.trainer_gpus}}\"}\n"
                         "      limits: {memory: \"{{workflow.parameters.trainer_ram}}Gi\", "
                         "cpu: \"{{workflow.parameters.trainer_cores}}\", "
                         "amd.com/gpu: \"{{workflow.parameters.trainer_gpus}}\"}\n"),
        "container": {
            "image": kca, "command": ["/bin/bash", "-c"],
            "args": ["python3 -m kubernetes_cloud_amd.launch --num_gpus {{workflow.parameters.trainer_gpus}} "
                     "-m kubernetes_cloud_amd.train.finetuner {{inputs.parameters.finetuner_params}}"],
            "env": [{"name": "WANDB_API_KEY", "value": ip("wandb_key")}] + list(ROCM_ENV),
            "resources": resources(gpus=1, cpu=16, memory="256Gi"),
            "volumeMounts": [_vol_mount(), {"name": "dshm", "mountPath": "/dev/shm"}]},
        "volumes": [pvc_volume(wp("pvc")), shm_volume()],
        "affinity": affinity(wp("trainer_gpu"), wp("region")),
    }
    isvc_manifest = {
        "apiVersion": "serving.kserve.io/v1beta1", "kind": "InferenceService",
        "metadata": {"name": "inference-{{ workflow.parameters.run_name }}",
                     "annotations": {"autoscaling.knative.dev/scaleToZeroPodRetentionPeriod": "20m"}},
        "spec": {"predictor": {
            "minReplicas": 0, "maxReplicas": 1, "affinity": affinity(wp("inference_gpu"), wp("region")),
            "containers": [{
                "name": "kserve-container", "image": kca, "imagePullPolicy": "IfNotPresent",
                "command": ["python3", "-m", "kubernetes_cloud_amd.serving.completion_server"],
                "args": ["--model=$(INFERENCE_MODEL)", "--port=$(INFERENCE_PORT)"],
                "env": [{"name": "INFERENCE_PORT", "value": "80"},
                        {"name": "INFERENCE_MODEL", "value": "/mnt/pvc/{{ inputs.parameters.model_path }}"},
                        {"name": "STORAGE_URI", "value": "pvc://{{ workflow.parameters.pvc }}/"}] + list(ROCM_ENV),
                "ports": [{"protocol": "TCP", "containerPort": 80}],
                "livenessProbe": {"httpGet": {"path": "/", "port": 80}, "initialDelaySeconds": 60, "periodSeconds": 30},
                "readinessProbe": {"httpGet": {"path": "/", "port": 80}, "initialDelaySeconds": 60,
                                   "periodSeconds": 30},
                "resources": {"requests": {"amd.com/gpu": 1, "cpu": 4, "memory": "16Gi"},
                              "limits": {"amd.com/gpu": 1, "cpu": 16, "memory": "128Gi"}}}]}}}
    import yaml
    isvc = {"name": "model-inference-service",
            "inputs": {"parameters": [{"name": "model_path"}, {"name": "model_name"}]},
            "resource": {"action": "apply", "manifest": yaml.safe_dump(isvc_manifest, sort_keys=False)}}
    return {"apiVersion": "argoproj.io/v1alpha1", "kind": "Workflow",
            "metadata": {"generateName": "finetune-"},
            "spec": {"entrypoint": "main", "serviceAccountName": "finetune",
                     "arguments": {"parameters": _params(FINETUNE_PARAMS)},
                     "templates": [main, check, dl, dsd, tok, ft, isvc]}}


# ------------------------------------------------------------ T10 / T11
SD_PARAMS = [
    ("run_name", None), ("pvc", "sd-finetune-data"), ("model", "stabilityai/stable-diffusion-2"),
    ("dataset", "dataset"), ("lr", "5e-6"), ("epochs", "10"), ("batch_size", "1"), ("use_ema", "False"),
    ("gradient_checkpointing", "False"), ("use_8bit_adam", "False"), ("adam_beta1", "0.9"),
    ("adam_beta2", "0.999"), ("adam_weight_decay", "1e-2"), ("adam_epsilon", "1e-8"), ("seed", "42"),
    ("save_steps", "500"), ("resolution", "512"), ("resize", "False"), ("center_crop", "False"),
    ("resize_interp", "lanczos"), ("shuffle", "True"), ("image_log_steps", "500"), ("image_log_amount", "4"),
    ("project_id", "sd-finetune"), ("use_tensorizer", True), ("run_inference", False), ("inference_only", False),
    ("region", "ORD1"), ("trainer_gpu", MI355X), ("trainer_gpu_count", "1"), ("inference_gpu", MI355X),
    ("downloader_image", "ghcr.io/kubernetes-cloud-amd/kca"), ("downloader_tag", "rocm7.2-gfx950"),
    ("finetuner_image", "ghcr.io/kubernetes-cloud-amd/kca"), ("finetuner_tag", "rocm7.2-gfx950"),
    ("serializer_image", "ghcr.io/kubernetes-cloud-amd/kca"), ("serializer_tag", "rocm7.2-gfx950"),
    ("inference_image", "ghcr.io/kubernetes-cloud-amd/kca"), ("inference_tag", "rocm7.2-gfx950"),
]

DB_PARAMS = [
    ("run_name", None), ("pvc", "db-finetune-data"), ("model", "stabilityai/stable-diffusion-2-1-base"),
    ("instance_dataset", "data/example-dog"), ("instance_prompt", "a photo of sks dog"), ("prior_loss_weight", 1.0),
    ("class_dataset", "generic/dogs-2"), ("class_prompt", "a photo of dog"), ("num_class_images", 100),
    ("output", "finetunes/example-dog"), ("lr", "2e-6"), ("lr_scheduler", "constant"), ("lr_warmup_steps", 0),
    ("batch_size", "1"), ("epochs", 4), ("seed", 42), ("checkpointing_steps", 200), ("image_log_steps", 100),
    ("image_log_amount", 4), ("resolution", "512"), ("use_tensorizer", True), ("run_inference", True),
    ("inference_only", False), ("region", "LAS1"), ("trainer_gpu", MI355X), ("trainer_gpu_count", "1"),
    ("inference_gpu", MI355X), ("downloader_image", "ghcr.io/kubernetes-cloud-amd/kca"),
    ("downloader_tag", "rocm7.2-gfx950"), ("finetuner_image", "ghcr.io/kubernetes-cloud-amd/kca"),
    ("finetuner_tag", "rocm7.2-gfx950"), ("serializer_image", "ghcr.io/kubernetes-cloud-amd/kca"),
    ("serializer_tag", "rocm7.2-gfx950"), ("inference_image", "ghcr.io/kubernetes-cloud-amd/kca"),
    ("inference_tag", "rocm7.2-gfx950"),
]

_SD_FT_FLAGS = ["run_name", "model", "dataset", "lr", "epochs", "batch_size", "use_ema", "gradient_checkpointing",
                "use_8bit_adam", "adam_beta1", "adam_beta2", "adam_weight_decay", "adam_epsilon", "seed",
                "output_path", "save_steps", "resolution", "resize", "center_crop", "resize_interp", "shuffle",
                "image_log_steps", "image_log_amount", "project_id"]
_DB_FT_FLAGS = [("run_name", "run_name"), ("model", "model"), ("instance_dataset", "instance_dataset"),
                ("class_dataset", "class_dataset"), ("instance_prompt", "instance_prompt"),
                ("class_prompt", "class_prompt"), ("num_class_images", "num_class_images"),
                ("output_path", "output_path"), ("prior_loss_weight", "prior_loss_weight"),
                ("resolution", "resolution"), ("batch_size", "batch_size"), ("lr", "lr"),
                ("lr_scheduler", "lr_scheduler"), ("lr_warmup_steps", "lr_warmup_steps"), ("epochs", "epochs"),
                ("save_steps", "checkpointing_steps"), ("image_log_steps", "image_log_steps"),
                ("image_log_amount", "image_log_amount"), ("seed", "seed")]


def _sd_template(name: str, params, dreambooth: bool) -> dict:
    pvc = wp("pvc")
    if dreambooth:
        out_path = "/" + pvc + "/" + wp("output")
        ft_inputs = [wf for _, wf in _DB_FT_FLAGS]
        ft_values = {wf: wp(wf) for wf in ft_inputs}
        ft_values.update(model="/" + pvc + "/models/" + wp("model"),
                         instance_dataset="/" + pvc + "/" + wp("instance_dataset"),
                         class_dataset="/" + pvc + "/" + wp("class_dataset"), output_path=out_path)
        ft_inputs = list(dict.fromkeys(ft_inputs + ["output_path"]))
        ft_values.pop("output", None)
        cli = []
        for flag, wf in _DB_FT_FLAGS:
            cli += ["--" + flag, ip(wf)]
        cli += ["--gradient_checkpointing", "true"]
        nproc = "1"  # DreamBooth pinned to one process (db-workflow-template.yaml:257-261)
    else:
        out_path = "/" + pvc + "/finetunes/" + wp("run_name")
        ft_inputs = list(_SD_FT_FLAGS)
        ft_values = {f: wp(f) for f in ft_inputs}
        ft_values.update(model="/" + pvc + "/models/" + wp("model"), dataset="/" + pvc + "/" + wp("dataset"),
                         output_path=out_path)
        cli = []
        for f in _SD_FT_FLAGS:
            cli += ["--" + f, ip(f)]
        nproc = ip("gpu_count")
        ft_inputs.append("gpu_count")
        ft_values["gpu_count"] = wp("trainer_gpu_count")
    kca_ft = image("finetuner_tag", "finetuner_image")
    main = {"name": "main", "steps": [
        [{"name": "downloader", "template": "model-downloader", "when": "{{workflow.parameters.inference_only}} == false",
          "arguments": {"parameters": [{"name": "model", "value": wp("model")},
                                       {"name": "dest", "value": "/" + pvc + "/models/" + wp("model")},
                                       {"name": "type", "value": "diffusers"}]}}],
        [{"name": "finetuner", "template": "model-finetuner", "when": "{{workflow.parameters.inference_only}} == false",
          "arguments": {"parameters": [{"name": k, "value": ft_values[k]} for k in ft_inputs]}}],
        [{"name": "serializer", "template": "serializer",
          "when": "{{workflow.parameters.use_tensorizer}} == true && {{workflow.parameters.inference_only}} == false",
          "arguments": {"parameters": [{"name": "model", "value": out_path}, {"name": "output_path", "value": out_path}]}}],
        [{"name": "inference", "template": "model-inference-service",
          "when": "{{workflow.parameters.run_inference}} == true || {{workflow.parameters.inference_only}} == true",
          "arguments": {"parameters": [{"name": "command", "value": (
              '["python3", "-m", "kubernetes_cloud_amd.serving.sd_service", "--model-id", "/mnt/pvc/'
              + (wp("output") if dreambooth else "finetunes/" + wp("run_name")) + '"'
              + '{{=workflow.parameters.use_tensorizer == "true" ? ", \\"--tensorized\\"" : ""}}]')}]}}],
    ]}
    dl = _cpu_step("model-downloader", ["model", "dest", "type"], image("downloader_tag", "downloader_image"),
                   ["python3", "-m", "kubernetes_cloud_amd.data.downloader"],
                   ["-model", ip("model"), "-dest", ip("dest"), "-type", ip("type")], cpu="4", mem="8Gi")
    ft = {"name": "model-finetuner", "inputs": {"parameters": [{"name": k} for k in ft_inputs]},
          "container": {
              "image": kca_ft,
              "command": ["python3", "-m", "kubernetes_cloud_amd.launch", "--num_gpus", nproc,
                          "-m", "kubernetes_cloud_amd.train.sd_finetuner"],
              "args": cli,
              "env": [{"name": "WANDB_API_KEY", "valueFrom": {"secretKeyRef": {"name": "wandb-token-secret",
                                                                                "key": "token", "optional": True}}},
                      {"name": "HUGGING_FACE_HUB_TOKEN", "valueFrom": {"secretKeyRef": {
                          "name": "huggingface-hub-token", "key": "token", "optional": True}}}] + list(ROCM_ENV),
              "resources": resources(gpus=(1 if dreambooth else wp("trainer_gpu_count")), cpu=16, memory="128Gi"),
              "volumeMounts": [_vol_mount(), {"name": "dshm", "mountPath": "/dev/shm"}]},
          "volumes": [pvc_volume(pvc), shm_volume()], "affinity": affinity(wp("trainer_gpu"), wp("region"))}
    ser = _cpu_step("serializer", ["model", "output_path"], image("serializer_tag", "serializer_image"),
                    ["python3", "-c", "from kubernetes_cloud_amd.serving.sd_service import serialize_main; "
                                      "serialize_main()"],
                    ["--model-id", ip("model"), "--save-path", ip("output_path")], cpu="8", mem="32Gi")
    import yaml
    isvc_manifest = {
        "apiVersion": "serving.kserve.io/v1beta1", "kind": "InferenceService",
        "metadata": {"name": f"{name}-{{{{workflow.parameters.run_name}}}}",
                     "annotations": {"autoscaling.knative.dev/scaleToZeroPodRetentionPeriod": "20m"}},
        "spec": {"predictor": {
            "containerConcurrency": 8, "minReplicas": 0, "maxReplicas": 1,
            "affinity": affinity(wp("inference_gpu"), wp("region")),
            "containers": [{"name": "kserve-container", "image": image("inference_tag", "inference_image"),
                            "command": "{{inputs.parameters.command}}",
                            "env": [{"name": "STORAGE_URI", "value": "pvc://" + pvc + "/"},
                                    {"name": "MAX_BATCH", "value": "8"}] + list(ROCM_ENV),
                            "resources": {"requests": {"amd.com/gpu": 1, "cpu": 4, "memory": "16Gi"},
                                          "limits": {"amd.com/gpu": 1, "cpu": 16, "memory": "64Gi"}}}]}}}
    isvc = {"name": "model-inference-service", "inputs": {"parameters": [{"name": "command"}]},
            "resource": {"action": "apply", "manifest": yaml.safe_dump(isvc_manifest, sort_keys=False)}}
    return {"apiVersion": "argoproj.io/v1alpha1", "kind": "WorkflowTemplate", "metadata": {"name": name},
            "spec": {"entrypoint": "main", "serviceAccountName": "inference",
                     "arguments": {"parameters": _params(params)}, "templates": [main, dl, ft, ser, isvc]}}


def sd_finetune_template() -> dict:
    return _sd_template("sd-finetune-template", SD_PARAMS, dreambooth=False)


def dreambooth_template() -> dict:
    return _sd_template("db-finetune-template", DB_PARAMS, dreambooth=True)


def event_binding(name: str, template: str, discriminator: str, payload: list[tuple]) -> dict:
    params = []
    for pname, expr in payload:
        params.append({"name": pname, "valueFrom": {"event": expr}})
    return {"apiVersion": "argoproj.io/v1alpha1", "kind": "WorkflowEventBinding", "metadata": {"name": name},
            "spec": {"event": {"selector": f'discriminator == "{discriminator}"'},
                     "submit": {"workflowTemplateRef": {"name": template}, "arguments": {"parameters": params}}}}


def sd_event_binding() -> dict:
    return event_binding("sd-finetune-event-binding", "sd-finetune-template", "sd-finetune", [
        ("run_name", "payload.run_name"), ("dataset", "payload.dataset"),
        ("run_inference", "payload.run_inference == null ? true : payload.run_inference"),
        ("inference_only", "payload.inference_only == null ? false : payload.inference_only")])


def db_event_binding() -> dict:
    return event_binding("db-finetune-event-binding", "db-finetune-template", "db-finetune", [
        ("run_name", "payload.run_name"), ("instance_dataset", "payload.instance_dataset"),
        ("instance_prompt", "payload.instance_prompt"), ("class_dataset", "payload.class_dataset"),
        ("class_prompt", "payload.class_prompt"), ("output", "payload.output"),
        ("num_class_images", "payload.num_class_images == null ? 100: payload.num_class_images"),
        ("run_inference", "payload.run_inference == null ? true : payload.run_inference"),
        ("inference_only", "payload.inference_only == null ? false : payload.inference_only")])


# ------------------------------------------------------------------ T12
NEOX_PARAMS = [
    ("run_name", None), ("pvc_data_name", "neox-data"), ("pvc_checkpoints_name", "neox-checkpoints"),
    ("download_checkpoint", True),
    ("model_weights_url", "https://the-eye.eu/public/AI/models/GPT-NeoX-20B/slim_weights/"),
    ("pretrained_checkpoint_path", "20B_pretrained_checkpoint"), ("finetuned_checkpoint_path", "20B_finetuned_checkpoint"),
    ("download_dataset", True), ("dataset_url", "https://the-eye.eu/public/AI/pile_preliminary_components/hn.tar.gz"),
    ("dataset_path", "datasets"), ("dataset_file", "hn.tar.gz"), ("tokenize_dataset", True),
    ("tokenized_dataset_path", "datasets/hackernews"), ("training_config_name", "neox-training"),
    ("region", "LAS1"), ("trainer_nodes", 1), ("trainer_gpu", MI355X), ("use_ib", False),
    ("micro_batch_size", 8), ("gradient_accumulation_steps", 96), ("tensor_parallel", 2), ("pipeline_parallel", 4),
    ("wandb_secret_name", "wandb-token-secret"), ("wandb_project", "finetune-gpt-neox"),
    ("wandb_group", "MI355X-1N"), ("downloader_image", "cirrusci/wget"), ("downloader_tag", "latest"),
    ("gpt_neox_image", "ghcr.io/kubernetes-cloud-amd/kca"), ("gpt_neox_tag", "rocm7.2-gfx950"),
]


def neox_workflow() -> dict:
    """GPT-NeoX-20B TP x PP x DP finetune as a PyTorchJob (torchrun per node,
    RCCL), replacing the MPIJob + external gpt-neox image of the reference."""
    import yaml
    pj = {
        "apiVersion": "kubeflow.org/v1", "kind": "PyTorchJob",
        "metadata": {"name": "neox-{{workflow.parameters.run_name}}"},
        "spec": {"pytorchReplicaSpecs": {"Worker": {
            "replicas": "{{workflow.parameters.trainer_nodes}}", "restartPolicy": "OnFailure",
            "template": {"spec": {
                "affinity": affinity(wp("trainer_gpu"), wp("region")),
                "containers": [{
                    "name": "pytorch", "image": image("gpt_neox_tag", "gpt_neox_image"),
                    "command": ["torchrun", "--nproc-per-node", "8", "--nnodes",
                                "{{workflow.parameters.trainer_nodes}}",
                                "-m", "kubernetes_cloud_amd.train.parallel_trainer"],
                    "args": ["--model", "/mnt/checkpoints/{{workflow.parameters.pretrained_checkpoint_path}}",
                             "--dataset", "/mnt/data/{{workflow.parameters.tokenized_dataset_path}}",
                             "--output-path", "/mnt/checkpoints/{{workflow.parameters.finetuned_checkpoint_path}}",
                             "--tp", "{{workflow.parameters.tensor_parallel}}",
                             "--pp", "{{workflow.parameters.pipeline_parallel}}",
                             "--micro-batch", "{{workflow.parameters.micro_batch_size}}",
                             "--gradients", "{{workflow.parameters.gradient_accumulation_steps}}",
                             "--zero-stage", "1", "--gradient-checkpointing", "--lr", "6e-5",
                             "--betas", "0.9", "0.95", "--max-grad-norm", "1.0", "--lr-schedule", "cosine"],
                    "env": [{"name": "WANDB_PROJECT", "value": wp("wandb_project")},
                            {"name": "WANDB_RUN_GROUP", "value": wp("wandb_group")},
                            {"name": "WANDB_API_KEY", "valueFrom": {"secretKeyRef": {
                                "name": wp("wandb_secret_name"), "key": "token", "optional": True}}}] + list(ROCM_ENV),
                    "resources": resources(gpus=8, cpu=96, memory="1536Gi"),
                    "volumeMounts": [{"name": "data", "mountPath": "/mnt/data"},
                                     {"name": "checkpoints", "mountPath": "/mnt/checkpoints"},
                                     {"name": "dshm", "mountPath": "/dev/shm"}]}],
                "volumes": [{"name": "data", "persistentVolumeClaim": {"claimName": wp("pvc_data_name")}},
                            {"name": "checkpoints",
                             "persistentVolumeClaim": {"claimName": wp("pvc_checkpoints_name")}},
                            shm_volume()]}}}}}}
    main = {"name": "main", "dag": {"tasks": [
        {"name": "download-checkpoint", "template": "downloader", "when": "{{workflow.parameters.download_checkpoint}}",
         "arguments": {"parameters": [{"name": "url", "value": wp("model_weights_url")},
                                      {"name": "dest", "value": "/mnt/checkpoints/" + wp("pretrained_checkpoint_path")},
                                      {"name": "claim", "value": wp("pvc_checkpoints_name")}]}},
        {"name": "download-dataset", "template": "downloader", "when": "{{workflow.parameters.download_dataset}}",
         "arguments": {"parameters": [{"name": "url", "value": wp("dataset_url")},
                                      {"name": "dest", "value": "/mnt/checkpoints/" + wp("dataset_path")},
                                      {"name": "claim", "value": wp("pvc_data_name")}]}},
        {"name": "tokenize-dataset", "template": "tokenize-dataset", "dependencies": ["download-dataset"],
         "when": "{{workflow.parameters.tokenize_dataset}}"},
        {"name": "finetune", "template": "finetune", "dependencies": ["download-checkpoint", "tokenize-dataset"]},
    ]}}
    downloader = {"name": "downloader", "inputs": {"parameters": [{"name": "url"}, {"name": "dest"}, {"name": "claim"}]},
                  "container": {"image": image("downloader_tag", "downloader_image"), "command": ["sh", "-c"],
                                "args": ["mkdir -p {{inputs.parameters.dest}} && cd {{inputs.parameters.dest}} && "
                                         "wget -q -r -np -nH --cut-dirs=5 -R 'index.html*' {{inputs.parameters.url}}"],
                                "volumeMounts": [{"name": "vol", "mountPath": "/mnt/checkpoints"}]},
                  "volumes": [{"name": "vol", "persistentVolumeClaim": {"claimName": ip("claim")}}]}
    tokenize = {"name": "tokenize-dataset",
                "container": {"image": image("gpt_neox_tag", "gpt_neox_image"),
                              "command": ["python3", "-m", "kubernetes_cloud_amd.data.tokenizer"],
                              "args": ["-tokenizer", "/mnt/checkpoints/" + wp("pretrained_checkpoint_path"),
                                       "-input", "/mnt/data/" + wp("dataset_path"),
                                       "-output", "/mnt/data/" + wp("tokenized_dataset_path") + ".tokens",
                                       "-context", "2048"],
                              "volumeMounts": [{"name": "data", "mountPath": "/mnt/data"},
                                               {"name": "checkpoints", "mountPath": "/mnt/checkpoints"}]},
                "volumes": [{"name": "data", "persistentVolumeClaim": {"claimName": wp("pvc_data_name")}},
                            {"name": "checkpoints", "persistentVolumeClaim": {"claimName": wp("pvc_checkpoints_name")}}]}
    finetune = {"name": "finetune", "resource": {
        "action": "create", "successCondition": "status.replicaStatuses.Worker.succeeded > 0",
        "failureCondition": "status.replicaStatuses.Worker.failed > 0",
        "manifest": yaml.safe_dump(pj, sort_keys=False)}}
    return {"apiVersion": "argoproj.io/v1alpha1", "kind": "Workflow", "metadata": {"generateName": "neox-finetune-"},
            "spec": {"entrypoint": "main", "serviceAccountName": "finetune",
                     "arguments": {"parameters": _params(NEOX_PARAMS)},
                     "templates": [main, downloader, tokenize, finetune]}}


# ------------------------------------------------------------------- P1
def gpu_say_workflow() -> dict:
    return {"apiVersion": "argoproj.io/v1alpha1", "kind": "Workflow", "metadata": {"generateName": "gpu-say"},
            "spec": {"entrypoint": "main", "activeDeadlineSeconds": 300, "ttlSecondsAfterFinished": 86400,
                     "arguments": {"parameters": [{"name": "messages", "value": '["Argo", "On", "MI355X"]'}]},
                     "templates": [
                         {"name": "main", "steps": [[{"name": "echo", "template": "gpu-echo",
                                                      "arguments": {"parameters": [{"name": "message",
                                                                                    "value": "{{item}}"}]},
                                                      "withParam": wp("messages")}]]},
                         {"name": "gpu-echo", "inputs": {"parameters": [{"name": "message"}]},
                          "retryStrategy": {"limit": 1},
                          "script": {"image": image(), "command": ["bash"],
                                     "source": "rocm-smi --showproductname --showmeminfo vram\n"
                                               "python3 -c 'import torch; print(torch.cuda.get_device_name(0))'\n"
                                               "echo \"Input was: {{inputs.parameters.message}}\"\n",
                                     "resources": {"requests": {"memory": "512Mi", "cpu": "500m"},
                                                   "limits": {"amd.com/gpu": 1}}},
                          "affinity": affinity(MI355X, None)}]}}


__all__ = ["finetune_workflow", "sd_finetune_template", "dreambooth_template", "sd_event_binding",
           "db_event_binding", "neox_workflow", "gpu_say_workflow", "FINETUNE_PARAMS", "SD_PARAMS", "DB_PARAMS",
           "NEOX_PARAMS"]
