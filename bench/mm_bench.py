#!/usr/bin/env python3
"""Batched-decode GEMM microbenchmark: the MFMA skinny kernel (ops/skinny_mm.py) vs hipBLASLt
(F.linear) vs the VALU skinny kernel, on the decode weights of the served models, M = 1..64.

Each case is captured into a HIP graph of 20 back-to-back launches (launch overhead out of the
picture, every launch streams a cold weight: 20 distinct copies rotate), replayed, timed with events.
One JSON line per (shape, M): us per launch and the weight stream rate (GB/s).
"""
from __future__ import annotations

import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch
import torch.nn.functional as F

SHAPES = {
    # name: (N, K)
    "gptj.qkv": (12288, 4096), "gptj.out": (4096, 4096), "gptj.fc_in": (16384, 4096), "gptj.fc_out": (4096, 16384),
    "bloom8.qkv": (5376, 14336), "bloom8.out": (14336, 1792), "bloom8.fc_in": (7168, 14336),
    "bloom8.fc_out": (14336, 7168),
    "gptj.qkv_fcin": (28672, 4096), "gptj.out_fcout": (4096, 20480),
    "neox.qkv": (18432, 6144), "neox.out": (6144, 6144), "neox.fc_in": (24576, 6144), "neox.fc_out": (6144, 24576),
}


def _time_graph(fn, reps=20, iters=10):
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for i in range(2):
            fn(i)
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for i in range(reps):
            fn(i)
    g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        g.replay()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / (iters * reps)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shapes", default=",".join(SHAPES))
    ap.add_argument("--ms", default="1,2,4,8,16,32,64")
    ap.add_argument("--dtype", default="bf16")
    ap.add_argument("--variants", default="mfma,blas,valu")
    ap.add_argument("--ks", type=int, default=None)
    ap.add_argument("--nr", type=int, default=None)
    args = ap.parse_args()
    from kubernetes_cloud_amd.ops import _lib
    from kubernetes_cloud_amd.ops import skinny_mm as sm
    _lib.require()
    dt = {"bf16": torch.bfloat16, "fp16": torch.float16}[args.dtype]
    dev = torch.device("cuda", 0)
    for name in args.shapes.split(","):
        N, K = SHAPES[name]
        nbytes = N * K * 2
        copies = max(2, min(20, (3 << 30) // nbytes))
        ws = [torch.randn(N, K, device=dev).to(dt) * 0.02 for _ in range(copies)]
        for M in (int(m) for m in args.ms.split(",")):
            x = torch.randn(M, K, device=dev).to(dt)
            y = torch.empty(M, N, device=dev, dtype=dt)
            rec = {"shape": name, "N": N, "K": K, "M": M, "dtype": args.dtype}
            for v in args.variants.split(","):
                if v == "mfma":
                    fn = lambda i: sm.launch([sm.job([sm.part(x, ws[i % copies])], N, y)], M, dt,  # noqa: E731
                                             ks=args.ks, nr=args.nr)
                elif v == "blas":
                    fn = lambda i: torch.matmul(x, ws[i % copies].t(), out=y)  # noqa: E731
                elif v == "valu":
                    if M > 16 or dt != torch.bfloat16:
                        continue
                    fn = lambda i: _lib.call("kca_skinny_gemm", x.data_ptr(), x.stride(0),  # noqa: E731
                                             ws[i % copies].data_ptr(), None, y.data_ptr(), y.stride(0), M, N, K, 0,
                                             _lib.stream())
                else:
                    raise ValueError(v)
                us = _time_graph(fn)
                rec[v + "_us"] = round(us, 2)
                rec[v + "_gbps"] = round(nbytes / us / 1e3, 0)
            print(json.dumps(rec), flush=True)
        del ws
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
