"""the KCA_DASSERT debug kernel library (KCA_DEBUG=1 ->
libkca_kernels_debug.so) runs a training step and a decode step with every
bounds/invariant check armed, and is the library actually mapped."""
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CODE = r"""
import torch
from kubernetes_cloud_amd.ops import _lib
from kubernetes_cloud_amd.models.causal_lm import build_model
from kubernetes_cloud_amd.models.config import LMConfig, PRESETS_HF
from kubernetes_cloud_amd.train.engine import TrainEngine
from kubernetes_cloud_amd.engine.llm_engine import LLMEngine, SamplingParams
assert _lib.DEBUG and _lib.KERNEL_LIB.endswith("libkca_kernels_debug.so"), _lib.KERNEL_LIB
cfg = dict(PRESETS_HF["gpt-j-6b"]); cfg.update(n_embd=256, n_layer=2, n_head=4, rotary_dim=32, vocab_size=512)
m = build_model(LMConfig.from_hf(cfg), device="cuda", dtype=torch.bfloat16, seed=0)
eng = TrainEngine(m, lr=1e-4)
ids = torch.randint(0, 512, (2, 128), device="cuda")
mask = torch.ones(2, 128, dtype=torch.bool); mask[1, 100:] = False
for _ in range(2):
    eng.train_batch([ids], lambda b: m(b, labels=b, kv_len=torch.tensor([128, 100], dtype=torch.int32)))
eng.remove_hooks(); m.eval()
reqs = LLMEngine(m, max_slots=4, max_len=256).generate([[1, 2, 3], [4, 5]], SamplingParams(max_new_tokens=8))
torch.cuda.synchronize()
maps = open("/proc/self/maps").read()
assert "libkca_kernels_debug.so" in maps and "libkca_kernels.so" not in maps
print("debug-ok", [len(r.output) for r in reqs])
"""


def test_debug_kernel_library_step_and_decode():
    lib = os.path.join(ROOT, "kubernetes_cloud_amd", "_lib", "libkca_kernels_debug.so")
    if not os.path.exists(lib):
        pytest.skip("debug library not built (python tools/build_ext.py --debug)")
    r = subprocess.run([sys.executable, "-c", CODE], cwd=ROOT, capture_output=True, text=True, timeout=240,
                       env=dict(os.environ, KCA_DEBUG="1", PYTHONPATH=ROOT))
    assert r.returncode == 0 and "debug-ok" in r.stdout, (r.stdout + r.stderr)[-3000:]
