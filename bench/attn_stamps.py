#!/usr/bin/env python3
"""Where a full-tile attention loop iteration spends its cycles: runs forward +
backward of one shape on the diagnostic kernel build (``python tools/build_ext.py
--stamps`` -> ab/libkca_kernels_stamps.so, loaded through KCA_KERNEL_LIB) and
prints the per-segment shares of the s_memtime sums the kernels add up per wave
(csrc/kernels/attention_tiled.hip, ASTAMP). The stamps' fences forbid overlaps
the real kernels have, so the shares locate the time; the lengths are not the
real kernels' (they run ~10 % longer).

    KCA_KERNEL_LIB=$PWD/ab/libkca_kernels_stamps.so python bench/attn_stamps.py --shape gptj
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch

from kubernetes_cloud_amd import ops
from kubernetes_cloud_amd.ops import _lib

SEGMENTS = {
    "fwd": (0, ["prologue (Q, tiles 0-1, S0)", "issue K/V loads", "S=QK^T (next tile) + softmax",
                "O+=PV", "LDS store + barrier", "epilogue (O, lse stores)"]),
    "dq": (16, ["prologue", "issue K/V loads", "S, dP MFMAs", "softmax / dS", "dQ MFMAs",
                "LDS store + barrier", "epilogue (dQ stores)"]),
    "fwd_w8": (48, ["pre-wait (prologue, skipped tiles)", "vmcnt wait + barrier", "LDS-DMA issue",
                    "S=QK^T MFMAs", "mask + softmax", "O+=PV", "epilogue"]),
    "dkdv": (32, ["prologue (K, V image)", "issue Q/dO loads", "S, dP MFMAs", "softmax / dS",
                  "dV, dK MFMAs", "LDS store + barrier", "epilogue (dK, dV stores)"]),
}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shape", default="gptj")
    ap.add_argument("--iters", type=int, default=5)
    a = ap.parse_args()
    from attn_bench import SHAPES  # noqa: E402  (bench/ is this script's directory)
    B, Sq, Sk, H, D, causal = SHAPES[a.shape]
    lib = _lib.require()
    fn = getattr(lib, "kca_attn_stamps", None)
    if fn is None:
        raise SystemExit("not the stamp build: KCA_KERNEL_LIB=ab/libkca_kernels_stamps.so")
    buf = (ctypes.c_ulonglong * 64)()
    q = torch.randn(B, Sq, H, D, device="cuda", dtype=torch.bfloat16, requires_grad=True)
    k = torch.randn(B, Sk, H, D, device="cuda", dtype=torch.bfloat16, requires_grad=True)
    v = torch.randn(B, Sk, H, D, device="cuda", dtype=torch.bfloat16, requires_grad=True)
    o = ops.flash_attention(q, k, v, causal=causal)
    g = torch.randn_like(o)
    o.backward(g)
    torch.cuda.synchronize()
    fn(buf, 1)
    for _ in range(a.iters):
        o = ops.flash_attention(q, k, v, causal=causal)
        o.backward(g)
    torch.cuda.synchronize()
    assert fn(buf, 0) == 0
    vals = list(buf)
    out = {"shape": a.shape, "B": B, "S": Sq, "H": H, "D": D, "causal": causal, "iters": a.iters}
    for kern, (base, names) in SEGMENTS.items():
        seg = vals[base:base + len(names)]
        waves = vals[base + 7]
        tot = sum(seg) or 1
        out[kern] = {"waves": waves, "cycles_per_wave": round(tot / max(waves, 1)),
                     "share": {n: round(x / tot, 4) for n, x in zip(names, seg)}}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
