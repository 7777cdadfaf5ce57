#!/usr/bin/env python3
"""Per-call time of the fused all-reduce tails that close BLOOM TP=8's row-parallel projections
(``parallel/custom_ar.py`` res_ln at batch 1, res_stats at batch > 1; csrc/comm/xgmi_allreduce.hip) on
a rank-local (world 1) instance -- the kernels bench/bloom_tp_bench.py's emulated rank runs 140 times
per token. 100 calls captured in one HIP graph (the decode step's launch mode), microseconds per call.

    python bench/ar_tail_bench.py [--n 14336] [--batches 1,8,32]
One JSON line per (kind, batch).
"""
from __future__ import annotations

import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch


def _graph_us(fn, calls=100, reps=5):
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(3):
            fn()
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(calls):
            fn()
    g.replay()
    torch.cuda.synchronize()
    best = float("inf")
    for _ in range(reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        g.replay()
        e1.record()
        torch.cuda.synchronize()
        best = min(best, e0.elapsed_time(e1) * 1e3 / calls)
    return best


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=14336)
    ap.add_argument("--batches", default="1,8,32")
    ap.add_argument("--dtype", default="bf16")
    a = ap.parse_args()
    from kubernetes_cloud_amd.ops import skinny_mm as smm
    from kubernetes_cloud_amd.parallel.custom_ar import XGMIAllReduce
    dt = {"bf16": torch.bfloat16, "fp16": torch.float16}[a.dtype]
    dev = torch.device("cuda", 0)
    ar = XGMIAllReduce(None, max_bytes=16 << 20, local=True)
    N = a.n
    g = torch.Generator(device=dev).manual_seed(0)
    gamma = torch.ones(N, device=dev, dtype=dt)
    beta = torch.zeros(N, device=dev, dtype=dt)
    bias = (0.1 * torch.randn(N, device=dev, generator=g)).to(dt)
    for B in (int(b) for b in a.batches.split(",")):
        y = torch.randn(B, N, device=dev, generator=g).to(dt)
        h = torch.randn(B, N, device=dev, generator=g).to(dt)
        h_out = torch.empty_like(h)
        if B == 1:
            xn = torch.empty_like(h)
            us = _graph_us(lambda: ar.res_ln(y.view(-1), bias, h.view(-1), h_out.view(-1), gamma, beta, 1e-5,
                                             xn.view(-1)))
            kind = "res_ln"
        else:
            st = smm.RowStatsBuf(B, N, dev)
            us = _graph_us(lambda: ar.res_stats(y, bias, h, h_out, st, 1e-5))
            kind = "res_stats"
        print(json.dumps({"kind": kind, "batch": B, "N": N, "dtype": a.dtype, "us_per_call": round(us, 2),
                          "ar_define": os.environ.get("KCA_AB_TAG", "")}), flush=True)
        assert ar.error() == 0
    ar.close()


if __name__ == "__main__":
    main()
