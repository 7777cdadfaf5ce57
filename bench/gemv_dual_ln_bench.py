#!/usr/bin/env python3
"""Timing of the fused decode tail (kca_gemv_dual_ln: GEMV(s) + residual + LayerNorm in one launch) at the
decode shapes it serves: GPT-J (out + fc_out, N 4096), GPT-NeoX-20B (N 6144, two LayerNorms) and a
BLOOM TP=8 rank (out-projection K 1792 and fc_out K 7168 at N 14336). HIP-graph replay of 50
back-to-back launches, weights rotated over 4 copies (each launch streams from HBM, not the MALL).
One JSON line per shape: us per launch and the weight stream's TB/s. (The round-5 geometry sweep
behind the shipped defaults: profiles/decode_launch_structure_ab_r5.txt.)"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch

SHAPES = {"gptj": (4096, 4096, 16384, False), "neox20b": (6144, 6144, 24576, True),
          "bloom_tp8_out": (14336, 1792, 0, False), "bloom_tp8_fc_out": (14336, 7168, 0, False)}


def main():
    from kubernetes_cloud_amd.ops import decode as dops
    dev = torch.device("cuda", 0)
    bf = dict(device=dev, dtype=torch.bfloat16)
    for name, (N, K1, K2, two) in SHAPES.items():
        x1 = torch.randn(1, K1, **bf)
        x2 = torch.randn(1, K2, **bf) if K2 else None
        reps = 4
        w1 = [torch.randn(N, K1, **bf) * 0.02 for _ in range(reps)]
        w2 = [torch.randn(N, K2, **bf) * 0.02 if K2 else None for _ in range(reps)]
        b, h = torch.randn(N, **bf), torch.randn(1, N, **bf)
        g, be = torch.randn(N, **bf), torch.randn(N, **bf)
        ypart = torch.empty(N, device=dev, dtype=torch.float32)
        cnt = torch.zeros(32 * 65, device=dev, dtype=torch.int32)
        ho, xn, xn2 = torch.empty(1, N, **bf), torch.empty(1, N, **bf), torch.empty(1, N, **bf)
        mb = (K1 + K2) * N * 2 / 1e6
        res = {"shape": name, "N": N, "K": K1 + K2, "mbytes": round(mb, 1)}

        def run(i):
            dops.gemv_dual_ln(x1, w1[i % reps], x2, w2[i % reps], b, h, g, be, 1e-5, ypart, cnt, ho, xn,
                              *((g, be, xn2) if two else (None, None, None)))
        for i in range(8):
            run(i)
        torch.cuda.synchronize()
        gr = torch.cuda.CUDAGraph()
        with torch.cuda.graph(gr):
            for i in range(50):
                run(i)
        gr.replay()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(4):
            gr.replay()
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) * 1e3 / 200
        res.update(us=round(us, 2), tbs=round(mb / us, 2))
        print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
