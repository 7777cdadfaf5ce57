"""Deploy manifests + auxiliary CLIs: rendered YAML parses, uses amd.com/gpu
and MI355X affinity only, keeps the reference workflows' parameter surfaces
and event payload mappings, and every ``python -m`` entrypoint it names
exists; the model downloader (local mirror + .ready.txt + tensorize) and the
ResNet-50 DDP trainer (synthetic data) run."""
import importlib
import os
import re

import pytest
import torch
import yaml

from kubernetes_cloud_amd.deploy import render, workflows

REF = "/root/reference"


def _all_docs(out):
    docs = {}
    for path in render.render(out):
        with open(path) as f:
            docs[os.path.relpath(path, out)] = list(yaml.safe_load_all(f))
    return docs


def test_render_and_gpu_resources(tmp_path):
    docs = _all_docs(str(tmp_path))
    assert len(docs) > 30
    text = "\n".join(open(os.path.join(tmp_path, p)).read() for p in docs)
    assert "nvidia.com/gpu" not in text and "gpu.nvidia.com" not in text
    assert "amd.com/gpu" in text and "MI355X" in text
    # every python -m module the manifests launch is importable
    mods = set(re.findall(r"-m[\"',\s]+(kubernetes_cloud_amd[\w.]+)", text))
    mods |= set(re.findall(r"from (kubernetes_cloud_amd[\w.]+) import (\w+)", text))
    assert mods
    for m in mods:
        if isinstance(m, tuple):
            assert hasattr(importlib.import_module(m[0]), m[1]), m
        else:
            importlib.import_module(m)


def _ref_params(path):
    out = []
    for d in yaml.safe_load_all(open(path)):
        if d and "spec" in d:
            out += [p["name"] for p in d["spec"].get("arguments", {}).get("parameters", [])]
    return out


@pytest.mark.skipif(not os.path.isdir(REF), reason="reference tree not mounted")
@pytest.mark.parametrize("ref,ours", [
    ("finetuner-workflow/finetune-workflow.yaml", workflows.FINETUNE_PARAMS),
    ("sd-finetuner-workflow/sd-finetune-workflow-template.yaml", workflows.SD_PARAMS),
    ("sd-dreambooth-workflow/db-workflow-template.yaml", workflows.DB_PARAMS),
    ("kubeflow/training-operator/gpt-neox/04-finetune-workflow.yaml", workflows.NEOX_PARAMS),
])
def test_workflow_parameter_surface(ref, ours):
    names = {n for n, _ in ours}
    missing = [p for p in _ref_params(os.path.join(REF, ref)) if p not in names]
    assert not missing, missing


def test_event_bindings_map_payloads():
    sd = workflows.sd_event_binding()
    assert sd["spec"]["submit"]["workflowTemplateRef"]["name"] == "sd-finetune-template"
    db = workflows.db_event_binding()
    keys = [p["name"] for p in db["spec"]["submit"]["arguments"]["parameters"]]
    assert keys[:3] == ["run_name", "instance_dataset", "instance_prompt"] and "num_class_images" in keys


def test_downloader_local_mirror(tmp_path):
    from kubernetes_cloud_amd.data.downloader import main
    from .helpers import make_model_dir
    src = make_model_dir(str(tmp_path / "src"), "gpt2")
    dst = str(tmp_path / "dst")
    main(["-model", src, "-dest", dst, "-ready", "-tensorize", "model.tensors", "-dtype", "float32"])
    assert os.path.exists(os.path.join(dst, ".ready.txt")) and os.path.exists(os.path.join(dst, "model.tensors"))
    tok = str(tmp_path / "tok")
    main(["-model", src, "-dest", tok, "-tokenizer-only", "true"])
    assert not any(f.endswith(".safetensors") for f in os.listdir(tok))
    out = tmp_path / "probe.txt"
    os.environ["TENSORIZED_BASE_URL"] = "http://127.0.0.1:9"
    main(["check-tensorized", "-model", "x/y", "-out", str(out)])
    assert out.read_text() == "false"


def test_resnet50_synthetic(tmp_path):
    from kubernetes_cloud_amd.models.resnet import resnet50
    from kubernetes_cloud_amd.train.resnet import main
    m = resnet50()
    assert sum(p.numel() for p in m.parameters()) == 25_557_032  # torchvision resnet50
    assert "layer4.2.bn3.running_var" in m.state_dict()
    r = main(["--synthetic", "8", "--batch-size", "4", "--epochs", "1", "--max-steps", "2", "-j", "0",
              "--train-crop-size", "64", "--val-crop-size", "64", "--num-classes", "10", "--log-dir",
              str(tmp_path / "logs"), "--model-dir", str(tmp_path / "ck"), "--no-cuda"])
    assert r["steps"] == 2 and os.path.exists(tmp_path / "ck" / "resnet50_imagenet.pt")
    sd = torch.load(tmp_path / "ck" / "resnet50_imagenet.pt", weights_only=True)
    assert sd["fc.weight"].shape == (10, 2048)
