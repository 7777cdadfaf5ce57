"""User-facing entry points on the MI355X: the causal-LM
finetuner CLI (tiny GPT-J, bf16, checkpoint-2, a killed run resumed, final/
with .ready.txt), the SD finetuner in DreamBooth mode (class images generated
on the GPU, diffusers layout written), and the SD / GPT-J (tensorized) KServe
predictors returning PNG bytes and text -- all through the native kernels."""
import io
import os
import subprocess
import sys

import numpy as np
import pytest
import torch

from .helpers import make_images, make_model_dir, make_sd_dir, make_tokens

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(argv, env_extra=None, timeout=300):
    env = dict(os.environ, PYTHONPATH=ROOT, **(env_extra or {}))
    return subprocess.run([sys.executable, "-u"] + argv, cwd=ROOT, env=env, capture_output=True, text=True,
                          timeout=timeout)


def test_finetuner_cli_checkpoint_kill_resume_final(tmp_path):
    from kubernetes_cloud_amd.io.hf import read_hf_state_dict
    model = make_model_dir(str(tmp_path / "m"), "gpt-j-6b", n_embd=256, n_head=4, rotary_dim=32, vocab_size=512)
    data = make_tokens(str(tmp_path / "d.tokens"), n_ctx=32, ctx=128, vocab=500)
    argv = ["-m", "kubernetes_cloud_amd.train.finetuner", "--run-name", "g", "--model", model, "--dataset", data,
            "--context-size", "128", "--bs", "2", "--gradients", "2", "--output-path", str(tmp_path / "o"),
            "--logs", str(tmp_path / "l"), "--save-steps", "2", "--max-steps", "4", "--zero-stage", "0"]
    # dies hard before step 3, once checkpoint-2's async write has landed (otherwise the kill can beat the
    # writer and the restart rightly starts over: the resume assertion below would depend on timing)
    r = _run(argv, {"KCA_FAULT_STEP": "3", "KCA_FAULT_RANKS": "0", "KCA_FAULT_AFTER_CKPT": "1"})
    assert r.returncode == 17, r.stderr[-3000:]
    rd = tmp_path / "o" / "results-g"
    assert (rd / "checkpoint-2" / "model.safetensors").exists() and not (rd / "final").exists()
    r = _run(argv)
    assert r.returncode == 0, r.stderr[-3000:]
    assert "RESUMED" in r.stderr
    assert (rd / "final" / ".ready.txt").exists() and (rd / "checkpoint-4").exists()
    fin = read_hf_state_dict(str(rd / "final"))
    src = read_hf_state_dict(model)
    assert all(torch.isfinite(v.float()).all() for v in fin.values())
    assert any(not torch.equal(fin[k].float(), src[k].float()) for k in src)  # it trained


def test_sd_finetuner_dreambooth_gpu(tmp_path):
    d = make_sd_dir(str(tmp_path / "sd"))
    inst = make_images(str(tmp_path / "inst"), 2, captions=False)
    out = tmp_path / "db"
    r = _run(["-m", "kubernetes_cloud_amd.train.sd_finetuner", "--model", d, "--run_name", "db",
              "--instance_dataset", inst, "--instance_prompt", "a sks fox", "--class_dataset",
              str(tmp_path / "cls"), "--class_prompt", "a fox", "--num_class_images", "2", "--resolution", "32",
              "--batch_size", "1", "--epochs", "1", "--output_path", str(out), "--image_log_steps", "0",
              "--use_ema", "True"], {"KCA_CLASS_IMAGE_STEPS": "4"})
    assert r.returncode == 0, r.stderr[-3000:]
    assert len([f for f in os.listdir(tmp_path / "cls") if f.endswith(".jpg")]) == 2
    for sub in ("unet/diffusion_pytorch_model.safetensors", "vae/diffusion_pytorch_model.safetensors",
                "text_encoder/model.safetensors", "model_index.json", "scheduler/scheduler_config.json"):
        assert (out / sub).exists(), sub


def test_sd_predictor_png_on_gpu(tmp_path):
    from PIL import Image

    from kubernetes_cloud_amd.serving.sd_service import SDPredictor, serialize_main
    d = make_sd_dir(str(tmp_path / "sd"))
    serialize_main(["--model-id", d, "--save-path", str(tmp_path / "tz")])
    p = SDPredictor(model_name="sd", model_id=str(tmp_path / "tz"), tensorized=True, num_inference_steps=4,
                    width=32, height=32, max_batch=4, batch_window_ms=20)
    p.load()
    assert next(p.pipeline.unet.parameters()).is_cuda
    req = {"prompt": "a fox", "parameters": {"seed": 3, "guidance_scale": 5}}
    png = p.predict(req)
    assert png[:8] == b"\x89PNG\r\n\x1a\n" and Image.open(io.BytesIO(png)).size == (32, 32)
    # default (fastest-solver) mode: MIOpen may pick split-K convolutions that accumulate through
    # atomics (utils/miopen.py), so a repeat can move a pixel by a rounding step, never more
    for _ in range(3):
        a = np.asarray(Image.open(io.BytesIO(png)), dtype=np.int16)
        b = np.asarray(Image.open(io.BytesIO(p.predict(req))), dtype=np.int16)
        assert np.abs(a - b).max() <= 3 and np.abs(a - b).mean() < 0.5


def test_sd_predictor_deterministic_png_on_gpu(tmp_path):
    """``--deterministic``: the same seed gives the same PNG bytes (run in a fresh process:
    the MIOpen solver policy is fixed at the first convolution)."""
    code = f"""
import sys
sys.path.insert(0, {os.path.join(ROOT, "tests")!r})
from helpers import make_sd_dir
from kubernetes_cloud_amd.serving.sd_service import SDPredictor, serialize_main
d = make_sd_dir({str(tmp_path / "sd")!r})
serialize_main(["--model-id", d, "--save-path", {str(tmp_path / "tz")!r}])
p = SDPredictor(model_name="sd", model_id={str(tmp_path / "tz")!r}, tensorized=True, num_inference_steps=4,
                width=32, height=32, max_batch=4, batch_window_ms=20, deterministic=True)
p.load()
req = {{"prompt": "a fox", "parameters": {{"seed": 3, "guidance_scale": 5}}}}
pngs = [p.predict(req) for _ in range(6)]
assert all(x == pngs[0] for x in pngs), [x == pngs[0] for x in pngs]
print("DETERMINISTIC_OK")
"""
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=300, cwd=ROOT,
                       env={**os.environ, "PYTHONPATH": ROOT})
    assert r.returncode == 0 and "DETERMINISTIC_OK" in r.stdout, r.stderr[-3000:]


def test_gptj_tensorized_predictor_on_gpu(tmp_path):
    from fastapi.testclient import TestClient

    from kubernetes_cloud_amd.io.hf import load_pretrained, serialize_causal_lm
    from kubernetes_cloud_amd.serving.predictors import GPTJPredictor
    from kubernetes_cloud_amd.serving.server import ModelServer
    d = make_model_dir(str(tmp_path / "gptj"), "gpt-j-6b", n_embd=256, n_head=4, rotary_dim=32)
    serialize_causal_lm(load_pretrained(d, dtype=torch.float16), os.path.join(d, "gptj.tensors"))
    p = GPTJPredictor(model_path=d, load_type="tensorizer")
    p.load()
    assert next(p.generator.model.parameters()).is_cuda
    c = TestClient(ModelServer(http_port=1).create_app([p]))
    r = c.post("/v1/models/gptj:predict", json={"instances": ["hello there", "kubernetes"]}).json()
    assert len(r["predictions"]) == 2 and r["predictions"][0].startswith("hello there")
    p.generator.close()
