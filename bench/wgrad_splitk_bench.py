#!/usr/bin/env python3
"""Weight-gradient GEMMs of the SD UNet linears (small output, long token K) on MI355X: one
hipBLASLt GEMM (dW = dY^T X) vs the same product split over token chunks as a batched GEMM
plus an fp32 sum of the partials."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from kubernetes_cloud_amd.utils import tunable

tunable.ensure(tunable.SD_FILE)


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


dev = torch.device("cuda", 0)
for (T, N, K) in [(65536, 320, 320), (16384, 640, 640), (4096, 1280, 1280), (65536, 2560, 320),
                  (65536, 320, 1280), (16384, 5120, 640), (16384, 640, 2560)]:
    dy = torch.randn(T, N, device=dev, dtype=torch.bfloat16)
    x = torch.randn(T, K, device=dev, dtype=torch.bfloat16)
    ref = dy.float().t() @ x.float()
    t1 = timeit(lambda: dy.t() @ x)
    rec = {"T": T, "N": N, "K": K, "mm_ms": round(t1, 4)}
    for S in (2, 4, 8, 16):
        if T % S:
            continue
        def f():
            return torch.bmm(dy.view(S, T // S, N).transpose(1, 2), x.view(S, T // S, K)).float().sum(0)
        t = timeit(f)
        err = float((f() - ref).abs().max() / ref.abs().max())
        rec[f"bmm{S}_ms"] = round(t, 4)
        rec[f"bmm{S}_err"] = round(err, 5)
    rec["mm_err"] = round(float(((dy.t() @ x).float() - ref).abs().max() / ref.abs().max()), 5)
    print(json.dumps(rec), flush=True)
