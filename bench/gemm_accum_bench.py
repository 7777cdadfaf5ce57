#!/usr/bin/env python3
"""Weight-gradient accumulation study (GPT-J shapes, one micro-batch of 16384
tokens): bf16 dW GEMM + ``kca_accum_grad`` into the fp32 flat buffer (what the
engine's post-accumulate hook does) vs one GEMM that accumulates straight into
the fp32 buffer (``addmm(..., out_dtype=float32, beta=1)``: hipBLASLt bf16
inputs with an fp32 C/D)."""
from __future__ import annotations

import json
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from kubernetes_cloud_amd.ops import _lib  # noqa: E402

T = 16384
SHAPES = {"qkv": (12288, 4096), "out": (4096, 4096), "fc_in": (16384, 4096), "fc_out": (4096, 16384),
          "qkv_fc_in": (28672, 4096), "out_fc_out": (4096, 20480)}


def timeit(fn, iters=20, warmup=5):
    for _ in range(warmup):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters


def main():
    _lib.require()
    dev = "cuda"
    for name, (N, K) in SHAPES.items():
        dyt = torch.randn(N, T, device=dev, dtype=torch.bfloat16)
        xt = torch.randn(K, T, device=dev, dtype=torch.bfloat16)
        acc = torch.zeros(N, K, device=dev, dtype=torch.float32)
        fl = 2.0 * T * N * K
        r = {"gemm": name, "N": N, "K": K, "T": T}

        def bf16_then_accum():
            dw = F.linear(dyt, xt)
            _lib.call("kca_accum_grad", acc.data_ptr(), dw.data_ptr(), 0.25, 0, dw.numel(), _lib.stream())

        r["bf16_gemm_ms"] = timeit(lambda: F.linear(dyt, xt))
        r["bf16_plus_accum_ms"] = timeit(bf16_then_accum)
        try:
            r["fp32_out_gemm_ms"] = timeit(lambda: torch.mm(dyt, xt.t(), out_dtype=torch.float32))
            r["fp32_addmm_accum_ms"] = timeit(
                lambda: torch.addmm(acc, dyt, xt.t(), out_dtype=torch.float32, beta=1.0, alpha=0.25, out=acc))
            ref = (dyt.float() @ xt.float().t())
            acc.zero_()
            torch.addmm(acc, dyt, xt.t(), out_dtype=torch.float32, beta=1.0, alpha=1.0, out=acc)
            r["fp32_addmm_rel_err"] = ((acc - ref).abs().max() / ref.abs().max()).item()
        except Exception as e:  # noqa: BLE001
            r["fp32_err"] = repr(e)[:300]
        for k in list(r):
            if k.endswith("_ms"):
                r[k.replace("_ms", "_tflops")] = round(fl / r[k] / 1e9, 1)
                r[k] = round(r[k], 4)
        print(json.dumps(r), flush=True)
        del dyt, xt, acc
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
