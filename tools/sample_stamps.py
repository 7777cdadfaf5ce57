#!/usr/bin/env python3
"""Where the multi-workgroup sampler (decode.hip sample_mwg_kernel) spends its time: per-segment
s_memtime sums of the diagnostic build (``python tools/build_ext.py --stamps`` ->
ab/libkca_kernels_stamps.so, loaded through KCA_KERNEL_LIB), per call, for one mode at B = 1.

    KCA_KERNEL_LIB=$PWD/ab/libkca_kernels_stamps.so python tools/sample_stamps.py --mode topk10
"""
import argparse
import ctypes
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from kubernetes_cloud_amd.ops import _lib
from kubernetes_cloud_amd.ops import decode as dops

SEG = {0: "chunk: load + penalties", 1: "chunk: max / sum / argmax", 2: "chunk: local k-th key (radix)",
       3: "chunk: candidate count + write", 4: "chunk: arrival (release, counter)", 8: "merge: partials + gather",
       9: "merge: barrier", 10: "merge: global k-th key (radix)", 11: "merge: top-p",
       12: "merge: multinomial + output"}
MODES = {"greedy": (0.0, 0, 1.0), "topk10": (1.0, 10, 1.0), "topk50": (1.0, 50, 1.0),
         "topk50_topp0.95": (1.0, 50, 0.95)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--modes", default="topk10,topk50_topp0.95")
    ap.add_argument("--calls", type=int, default=200)
    a = ap.parse_args()
    lib = _lib.require()
    fn = lib.kca_sample_stamps
    fn.argtypes, fn.restype = [ctypes.c_void_p, ctypes.c_int], ctypes.c_int
    dev = torch.device("cuda", 0)
    V = 50400
    logits = (torch.randn(1, V, device=dev) * 4).to(torch.bfloat16)
    for mode in a.modes.split(","):
        t, k, p = MODES[mode]
        f = lambda v, dt: torch.full((1,), v, dtype=dt, device=dev)  # noqa: E731
        kw = dict(temperature=f(t, torch.float32), top_k=f(k, torch.int32), top_p=f(p, torch.float32),
                  rep_penalty=f(1.0, torch.float32), seeds=torch.arange(1, device=dev))
        for _ in range(5):
            dops.sample_logits(logits, **kw)
        torch.cuda.synchronize()
        fn(None, 1)
        for _ in range(a.calls):
            dops.sample_logits(logits, **kw)
        torch.cuda.synchronize()
        buf = (ctypes.c_ulonglong * 16)()
        fn(ctypes.addressof(buf), 0)
        n = max(buf[15], 1)
        tot = sum(buf[i] for i in SEG)
        print(f"{mode}: {buf[15]} merges")
        for i, name in SEG.items():
            print(f"  {name:36s} {buf[i] / n:10.0f} ticks/call  {100 * buf[i] / max(tot, 1):5.1f} %")


if __name__ == "__main__":
    main()
