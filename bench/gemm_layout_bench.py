#!/usr/bin/env python3
"""GPT-J GEMM layout study on MI355X: the weight-gradient (dW = dY^T X, reduction
over tokens) and input-gradient (dX = dY W) GEMMs as PyTorch issues them (NT / NN:
neither operand K-contiguous) vs the same math on transposed operands so that
both are K-contiguous (TN, the layout the forward GEMMs run at ~2 PFLOP/s),
plus the cost of producing the transposed copies."""
from __future__ import annotations

import argparse
import json

import torch
import torch.nn.functional as F

T = 16384  # micro-batch 8 x seq 2048
SHAPES = {"qkv": (12288, 4096), "out": (4096, 4096), "fc_in": (16384, 4096), "fc_out": (4096, 16384)}


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
    ap = argparse.ArgumentParser()
    ap.add_argument("--tokens", type=int, default=T)
    a = ap.parse_args()
    dev = "cuda"
    for name, (N, K) in SHAPES.items():
        x = torch.randn(a.tokens, K, device=dev, dtype=torch.bfloat16)
        dy = torch.randn(a.tokens, N, device=dev, dtype=torch.bfloat16)
        w = torch.randn(N, K, device=dev, dtype=torch.bfloat16) * 0.02
        fl = 2.0 * a.tokens * N * K
        r = {"gemm": name, "N": N, "K": K, "T": a.tokens}
        r["fwd_tn_ms"] = timeit(lambda: F.linear(x, w))
        r["wgrad_nt_ms"] = timeit(lambda: dy.t() @ x)
        dyt, xt = dy.t().contiguous(), x.t().contiguous()
        r["wgrad_tn_ms"] = timeit(lambda: F.linear(dyt, xt))
        r["transpose_dy_ms"] = timeit(lambda: dy.t().contiguous())
        r["transpose_x_ms"] = timeit(lambda: x.t().contiguous())
        r["dgrad_nn_ms"] = timeit(lambda: dy @ w)
        wt = w.t().contiguous()
        r["dgrad_tn_ms"] = timeit(lambda: F.linear(dy, wt))
        for k in list(r):
            if k.endswith("_ms") and not k.startswith("transpose"):
                r[k.replace("_ms", "_tflops")] = round(fl / r[k] / 1e9, 1)
            if k.endswith("_ms"):
                r[k] = round(r[k], 4)
        err = (F.linear(dyt, xt).float() - (dy.t() @ x).float()).abs().max().item()
        r["wgrad_max_abs_diff"] = err
        print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
