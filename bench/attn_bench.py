#!/usr/bin/env python3
"""Attention micro-benchmark: native gfx950 flash attention vs torch SDPA.

Shapes: GPT-J training (B8 H16 S2048 D256 causal), NeoX-20B (H64 D96),
GPT-2 (H12 D64), BLOOM shard (H14 D128), SD-1.5 self-attn (S4096 D40 / 1024 D80)
and the SD cross-attention (K/V len 77). Reports ms and TFLOP/s (causal FLOPs
counted as half) for forward and forward+backward.
"""
from __future__ import annotations

import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch
import torch.nn.functional as F

from kubernetes_cloud_amd import ops

SHAPES = {
    "gptj": (8, 2048, 2048, 16, 256, True),
    "neox20b": (4, 2048, 2048, 64, 96, True),
    "pythia2.8b": (8, 2048, 2048, 32, 80, True),
    "gpt2": (16, 1024, 1024, 12, 64, True),
    "bloom_tp8": (4, 2048, 2048, 14, 128, True),
    "sd_64": (16, 4096, 4096, 8, 40, False),
    "sd_64_pad64": (16, 4096, 4096, 8, 64, False),  # SD heads zero-padded 40 -> 64 (UNet training path)
    "sd_64_pad48": (16, 4096, 4096, 8, 48, False),  # 40 -> 48 narrow storage (UNet inference path; fwd only)
    "sd_32": (16, 1024, 1024, 8, 80, False),
    "sd_32_pad96": (16, 1024, 1024, 8, 96, False),  # 80 -> 96 (UNet padding onto the D=96 full-tile kernels)
    "sd_16": (16, 256, 256, 8, 160, False),
    "d160_1k": (16, 1024, 1024, 8, 160, False),
    "d160_4k": (4, 4096, 4096, 8, 160, True),  # SD-1.5 1280-channel heads (native D=160 full tiles)
    "sd_cross": (16, 4096, 77, 8, 40, False),
    # the UNet inference call: 40 real dims stored 48 wide, V column 40 = 1 (row sums on the MFMA) ...
    "sd_64_pad48_rs": (16, 4096, 4096, 8, 48, False, "rowsum"),
    # ... and K pre-scaled with column 40 = 1 (softmax offset in the S MFMA, attention_tiled.hip MC)
    "sd_64_pad48_mc": (16, 4096, 4096, 8, 48, False, "maxcol"),
}


def timeit(fn, iters=10, warmup=3):
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


def run(name, B, Sq, Sk, H, D, causal, mode="", sdpa=True, bwd=True):
    import math
    dev = "cuda"
    q = torch.randn(B, Sq, H, D, device=dev, dtype=torch.bfloat16, requires_grad=True)
    k = torch.randn(B, Sk, H, D, device=dev, dtype=torch.bfloat16, requires_grad=True)
    v = torch.randn(B, Sk, H, D, device=dev, dtype=torch.bfloat16, requires_grad=True)
    flops = 4.0 * B * H * Sq * Sk * D * (0.5 if causal else 1.0)
    out = {"shape": name, "B": B, "Sq": Sq, "Sk": Sk, "H": H, "D": D, "causal": causal}
    kw = {}
    if mode:  # fwd-only inference variants on 40 real dims
        bwd = sdpa = False
        with torch.no_grad():
            for t in (q, k, v):
                t[..., 40:] = 0
            v[..., 40] = 1.0
            kw = dict(rowsum_col=40, scale=40 ** -0.5)
            if mode == "maxcol":
                k[..., :40] *= 40 ** -0.5 * math.log2(math.e)
                k[..., 40] = 1.0
                kw.update(max_col=40, scale=math.log(2.0))

    def f_fwd():
        with torch.no_grad():
            ops.flash_attention(q, k, v, causal=causal, **kw)

    if not bwd:
        t = timeit(f_fwd)
        out["native_fwd_ms"] = round(t, 3)
        out["native_fwd_tflops"] = round(flops / t / 1e9, 1)
        return out
    o = ops.flash_attention(q, k, v, causal=causal)
    g = torch.randn_like(o)

    def f_fb():
        o = ops.flash_attention(q, k, v, causal=causal)
        o.backward(g)

    t = timeit(f_fwd)
    out["native_fwd_ms"] = round(t, 3)
    out["native_fwd_tflops"] = round(flops / t / 1e9, 1)
    if bwd:
        t2 = timeit(f_fb)
        out["native_fwdbwd_ms"] = round(t2, 3)
        out["native_fwdbwd_tflops"] = round(3.5 * flops / t2 / 1e9, 1)
    if sdpa:
        qt, kt, vt = (x.detach().transpose(1, 2).contiguous().requires_grad_() for x in (q, k, v))
        try:
            def s_fwd():
                with torch.no_grad():
                    F.scaled_dot_product_attention(qt, kt, vt, is_causal=causal)
            t = timeit(s_fwd)
            out["sdpa_fwd_ms"] = round(t, 3)
            out["sdpa_fwd_tflops"] = round(flops / t / 1e9, 1)
            if bwd:
                og = torch.randn(B, H, Sq, D, device=dev, dtype=torch.bfloat16)

                def s_fb():
                    o = F.scaled_dot_product_attention(qt, kt, vt, is_causal=causal)
                    o.backward(og)
                t2 = timeit(s_fb)
                out["sdpa_fwdbwd_ms"] = round(t2, 3)
                out["sdpa_fwdbwd_tflops"] = round(3.5 * flops / t2 / 1e9, 1)
        except Exception as e:  # pragma: no cover
            out["sdpa_error"] = str(e)[:200]
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shapes", default=",".join(SHAPES))
    ap.add_argument("--no-sdpa", action="store_true")
    ap.add_argument("--fwd-only", action="store_true")
    ap.add_argument("--generic", action="store_true", help="disable the full-tile fast kernels")
    ap.add_argument("--variant", type=int, default=-1, help="kca_attn_set_variant bits (A/B); -1 = default")
    a = ap.parse_args()
    if a.variant >= 0:
        from kubernetes_cloud_amd.ops.attention import set_variant
        set_variant(a.variant)
    if a.generic:
        from kubernetes_cloud_amd.ops.attention import set_tiled_path
        set_tiled_path(False)
    for n in a.shapes.split(","):
        r = run(n, *SHAPES[n], sdpa=not a.no_sdpa, bwd=not a.fwd_only)
        print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
