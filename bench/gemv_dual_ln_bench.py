#!/usr/bin/env python3
"""Sweep of the fused decode tail (kca_gemv_dual_ln) over rows per workgroup and launch variants (bit 0:
grid capped at one residency round, row groups looped; bit 1: the two weight streams as two loops
instead of one K range) at the decode shapes it
serves: GPT-J (out + fc_out, N 4096), GPT-NeoX-20B (N 6144, two LayerNorms) and a BLOOM TP=8 rank
(out-projection K 1792 and fc_out K 7168 at N 14336). HIP-graph replay of 50 back-to-back launches
per arm, weights larger than the MALL between arms (cold-ish stream). One JSON line per shape."""
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
        reps = 4  # distinct weight copies, rotated: each launch streams from HBM, not the MALL
        w1 = [torch.randn(N, K1, **bf) * 0.02 for _ in range(reps)]
        w2 = [torch.randn(N, K2, **bf) * 0.02 if K2 else None for _ in range(reps)]
        b, h = torch.randn(N, **bf), torch.randn(1, N, **bf)
        g, be = torch.randn(N, **bf), torch.randn(N, **bf)
        ypart = torch.empty(N, device=dev, dtype=torch.float32)
        cnt = torch.zeros(32 * 65, device=dev, dtype=torch.int32)
        ho, xn, xn2 = torch.empty(1, N, **bf), torch.empty(1, N, **bf), torch.empty(1, N, **bf)
        res = {"shape": name, "N": N, "K": K1 + K2, "mbytes": round((K1 + K2) * N * 2 / 1e6, 1)}
        arms = [(4, v) for v in (0, 1, 2, 3, 4, 6)] + [(8, 0), (16, 0)]  # v 4 / 6: no tail (timing only)
        for rows, var in arms:
            def run(i):
                dops.gemv_dual_ln(x1, w1[i % reps], x2, w2[i % reps], b, h, g, be, 1e-5, ypart, cnt, ho, xn,
                                  *((g, be, xn2) if two else (None, None, None)), rows=rows, variant=var)
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
            res[f"r{rows}v{var}_us"] = round(us, 2)
        print(json.dumps(res), flush=True)


def attn_out_ab():
    """BLOOM TP=8 rank layer, batch 1, 160 cached tokens: attention -> out-projection -> residual + ln_2
    as one launch (decode_attn_out_ln) against decode_prep_attention + gemv_dual_ln."""
    from kubernetes_cloud_amd.ops import decode as dops
    dev = torch.device("cuda", 0)
    bf = dict(device=dev, dtype=torch.bfloat16)
    H, D, L, N, L0 = 14, 128, 512, 14336, 160
    kc = torch.randn(2, H, L, D, **bf)
    vc = torch.randn_like(kc)
    qkv = torch.randn(1, 3 * H * D, **bf)
    slots = torch.tensor([1], device=dev, dtype=torch.int32)
    pos = torch.tensor([L0 - 1], device=dev, dtype=torch.int32)
    kv_lens = pos + 1
    al = torch.rand(H, device=dev) * 0.5
    reps = 4
    ows = [torch.randn(N, H * D, **bf) * 0.02 for _ in range(reps)]
    ob, h, g, be = torch.randn(N, **bf), torch.randn(1, N, **bf), torch.randn(N, **bf), torch.randn(N, **bf)
    ws = torch.zeros(max(dops.decode_ws_floats(1, H, H, D, L), 1), device=dev, dtype=torch.float32)
    ypart = torch.empty(N, device=dev, dtype=torch.float32)
    cnt = torch.zeros(32 * 65, device=dev, dtype=torch.int32)
    done = torch.zeros(32, device=dev, dtype=torch.int32)
    out, ho, xn = torch.empty(1, H * D, **bf), torch.empty(1, N, **bf), torch.empty(1, N, **bf)
    res = {"shape": "bloom_tp8_attn_out_ln", "kv": L0}
    for fused in (False, True):
        def run(i):
            if fused:
                assert dops.decode_attn_out_ln(qkv, H, H, D, 0, False, None, None, pos, slots, kc, vc, kv_lens, L0,
                                               D ** -0.5, al, out, ws, None, 0, 0, ows[i % reps], ob, h, g, be, 1e-5,
                                               ypart, cnt, ho, xn, done)
            else:
                dops.decode_prep_attention(qkv, H, H, D, 0, False, None, None, pos, slots, kc, vc, kv_lens, L0,
                                           D ** -0.5, al, out=out, ws=ws)
                dops.gemv_dual_ln(out, ows[i % reps], None, None, ob, h, g, be, 1e-5, ypart, cnt, ho, xn)
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
        res["fused_us" if fused else "two_launch_us"] = round(e0.elapsed_time(e1) * 1e3 / 200, 2)
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
    attn_out_ab()
