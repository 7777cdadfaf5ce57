#!/usr/bin/env python3
"""Decode GEMM microbench: kca_skinny_gemm vs hipBLASLt (F.linear), achieved
weight-streaming bandwidth, GPT-J and BLOOM-TP8 decode shapes."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import torch.nn.functional as F

from kubernetes_cloud_amd.ops.gemv import skinny_linear

SHAPES = {"gptj_qkv": (12288, 4096), "gptj_out": (4096, 4096), "gptj_fc_in": (16384, 4096),
          "gptj_fc_out": (4096, 16384), "bloom8_qkv": (5376, 14336), "bloom8_out": (14336, 1792),
          "bloom8_fc_in": (7168, 14336), "bloom8_fc_out": (14336, 7168), "gptj_lm_head": (50400, 4096)}


def t(fn, it=50):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(it):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / it * 1e3  # us


def main():
    dev = torch.device("cuda", 0)
    for name, (N, K) in SHAPES.items():
        w = torch.randn(N, K, device=dev).to(torch.bfloat16)
        for M in (1, 4, 16):
            x = torch.randn(M, K, device=dev).to(torch.bfloat16)
            us_s = t(lambda: skinny_linear(x, w))
            us_b = t(lambda: F.linear(x, w))
            gb = N * K * 2 / 1e9
            print(json.dumps({"shape": name, "M": M, "N": N, "K": K, "skinny_us": round(us_s, 1),
                              "hipblaslt_us": round(us_b, 1), "skinny_TBps": round(gb / us_s * 1e3, 2),
                              "hipblaslt_TBps": round(gb / us_b * 1e3, 2)}), flush=True)


if __name__ == "__main__":
    main()
