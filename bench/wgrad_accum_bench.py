"""Weight-gradient GEMM + fp32 accumulation: two ways, GPT-J shapes (mb16 x 2048 tokens).

  split : dW = F.linear(dY^T, X^T) in bf16 (TN, TunableOp table) then kca_accum_grad into fp32
  fused : torch.addmm(acc, dY^T, X, beta=1, alpha=scale, out_dtype=float32, out=acc) -- hipBLASLt
          reads the fp32 accumulator as C and writes D = C + scale * A B in place

Prints ms per call and the fp32 result error against the split path. Used to decide whether the
training engine's gradient sink may hand the GEMM its fp32 buffer directly (train/engine.py).
"""
from __future__ import annotations

import argparse
import json
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from kubernetes_cloud_amd.ops import _lib  # noqa: E402

SHAPES = {"qkv": (12288, 4096), "out": (4096, 4096), "fc_in": (16384, 4096), "fc_out": (4096, 16384)}


def timed(fn, iters):
    st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fn()
    torch.cuda.synchronize()
    st.record()
    for _ in range(iters):
        fn()
    en.record()
    torch.cuda.synchronize()
    return st.elapsed_time(en) / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tokens", type=int, default=32768)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--layer-gemms", action="store_true",
                    help="also time the block's forward / data-grad GEMMs (TN, as ops/fused_block.py issues them)")
    ap.add_argument("--tunableop", default=os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                                         "tuning", "tunableop_results.csv"))
    args = ap.parse_args()
    if args.tunableop and os.path.exists(args.tunableop):
        import torch.cuda.tunable as tunable
        tunable.enable(True)
        tunable.set_filename(args.tunableop, insert_device_ordinal=False)
        tunable.tuning_enable(False)
        tunable.read_file(args.tunableop)
    _lib.require()
    dev = torch.device("cuda")
    T = args.tokens
    for name, (n, k) in SHAPES.items():
        dyt = torch.randn(n, T, device=dev, dtype=torch.bfloat16)  # dY^T (transposed once, as in the block)
        xt = torch.randn(k, T, device=dev, dtype=torch.bfloat16)  # X^T
        acc0 = torch.randn(n, k, device=dev, dtype=torch.float32)
        acc_s, acc_f = acc0.clone(), acc0.clone()
        scale = 0.5

        def split():
            g = F.linear(dyt, xt)
            _lib.call("kca_accum_grad", acc_s.data_ptr(), g.data_ptr(), scale, 0, g.numel(), _lib.stream())

        def fused():
            torch.addmm(acc_f, dyt, xt.t(), beta=1.0, alpha=scale, out_dtype=torch.float32, out=acc_f)

        acc_s.copy_(acc0)
        acc_f.copy_(acc0)
        split()
        fused()
        torch.cuda.synchronize()
        ref = acc0 + scale * (dyt.float() @ xt.float().t())
        e_s = ((acc_s - ref).abs().max() / ref.abs().max()).item()
        e_f = ((acc_f - ref).abs().max() / ref.abs().max()).item()
        t_s = timed(split, args.iters)
        t_f = timed(fused, args.iters)
        fl = 2.0 * n * k * T
        print(json.dumps({"gemm": name, "n": n, "k": k, "tokens": T, "split_ms": round(t_s, 3),
                          "fused_ms": round(t_f, 3), "split_pf": round(fl / t_s / 1e12, 3),
                          "fused_pf": round(fl / t_f / 1e12, 3), "err_split": e_s, "err_fused": e_f}), flush=True)
        del dyt, xt, acc0, acc_s, acc_f, ref
        torch.cuda.empty_cache()
    if args.layer_gemms:
        for name, (n, k) in SHAPES.items():
            x = torch.randn(T, k, device=dev, dtype=torch.bfloat16)
            w = torch.randn(n, k, device=dev, dtype=torch.bfloat16)
            dy = torch.randn(T, n, device=dev, dtype=torch.bfloat16)
            wt = w.t().contiguous()
            fl = 2.0 * n * k * T
            t_f = timed(lambda: F.linear(x, w), args.iters)
            t_d = timed(lambda: F.linear(dy, wt), args.iters)
            print(json.dumps({"gemm": name, "fwd_ms": round(t_f, 3), "fwd_pf": round(fl / t_f / 1e12, 3),
                              "dgrad_ms": round(t_d, 3), "dgrad_pf": round(fl / t_d / 1e12, 3)}), flush=True)
            del x, w, dy, wt
            torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
