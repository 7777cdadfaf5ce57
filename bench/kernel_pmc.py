#!/usr/bin/env python3
"""Counter-profiling driver for the framework's hand-written gfx950 kernels.

Runs every hot native kernel a fixed number of times on the shape it sees in
the flagship workloads (GPT-J-6B training, SD-1.5 UNet, GPT-J decode), with a
kernel-name marker in stdout, so that one ``rocprofv3 --pmc`` pass per counter
group collects per-dispatch counters for all of them.  ``tools/pmc_summary.py``
joins the passes and derives MFMA utilisation, wave-state shares, LDS bank
conflict rate and HBM bandwidth per kernel; ``tools/pmc_profile.sh`` is the
recipe.  FLOP/byte models for each case are written to
``gpurun_out/pmc/cases.json`` so the summary can price them.

Shapes: K2 GPT-J attention B8 S2048 H16 D256 causal, K16 SD
self-attention B16 S4096 H8 D40, K4 LayerNorm 16384x4096, K14 NHWC GroupNorm
[8,320,64,64] +SiLU, K17 GEGLU 32768x(2x1280), K6 cross-entropy 16384x50400,
K7 AdamW over 512M fp32 params, skinny decode GEMV (GPT-J fc_in at M=1),
K12 decode attention (GPT-J B32, 2048 cached tokens).
"""
from __future__ import annotations

import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from kubernetes_cloud_amd import ops  # noqa: E402
from kubernetes_cloud_amd.ops import _lib  # noqa: E402

DEV = torch.device("cuda", 0)
BF = torch.bfloat16


def _attn(B, S, H, D, causal):
    q = torch.randn(B, S, H, D, device=DEV, dtype=BF, requires_grad=True)
    k = torch.randn(B, S, H, D, device=DEV, dtype=BF, requires_grad=True)
    v = torch.randn(B, S, H, D, device=DEV, dtype=BF, requires_grad=True)
    do = torch.randn(B, S, H, D, device=DEV, dtype=BF)

    def run():
        o = ops.flash_attention(q, k, v, causal=causal)
        o.backward(do)
        q.grad = k.grad = v.grad = None

    f = 4.0 * B * H * S * S * D * (0.5 if causal else 1.0)
    # fwd kernel: f; backward (dq + dkdv kernels): 2.5 f
    return run, {"fwd_flops": f, "bwd_flops": 2.5 * f}


def _attn_sd_tiled(B, S, H, hd, dp):
    """The DreamBooth UNet self-attention as it runs in training (models/unet.py Attention.forward): one
    fused [B, S, 3*H*dp] QKV buffer whose 40-wide heads are stored 48 wide (zero columns 40..47), the
    narrow-storage tiled kernels (attention_tiled.hip StagerNarrow, DS = 48 in the D = 64 LDS images)."""
    q5 = torch.randn(B, S, 3, H, dp, device=DEV, dtype=BF)
    q5[..., hd:] = 0
    qkv = q5.view(B, S, 3 * H * dp).requires_grad_(True)
    do = torch.randn(B, S, H * dp, device=DEV, dtype=BF)
    do.view(B, S, H, dp)[..., hd:] = 0

    def run():
        o = ops.qkv_rope_attention(qkv, H, dp, 0, False, causal=False, scale=hd ** -0.5)
        o.backward(do)
        qkv.grad = None

    f = 4.0 * B * H * S * S * hd
    return run, {"fwd_flops": f, "bwd_flops": 2.5 * f}


def _layernorm(rows, d):
    x = torch.randn(rows, d, device=DEV, dtype=BF, requires_grad=True)
    w = torch.randn(d, device=DEV, dtype=BF, requires_grad=True)
    b = torch.randn(d, device=DEV, dtype=BF, requires_grad=True)
    dy = torch.randn(rows, d, device=DEV, dtype=BF)

    def run():
        y = ops.layer_norm(x, w, b, 1e-5)
        y.backward(dy)
        x.grad = w.grad = b.grad = None

    return run, {"fwd_bytes": 2 * rows * d * 2, "bwd_bytes": 3 * rows * d * 2}


def _groupnorm(n, c, h, w_):
    x = torch.randn(n, c, h, w_, device=DEV, dtype=BF).to(memory_format=torch.channels_last)
    x.requires_grad_()
    w = torch.randn(c, device=DEV, dtype=BF, requires_grad=True)
    b = torch.randn(c, device=DEV, dtype=BF, requires_grad=True)
    dy = torch.randn(n, c, h, w_, device=DEV, dtype=BF).to(memory_format=torch.channels_last)

    def run():
        y = ops.group_norm(x, 32, w, b, 1e-5, silu=True)
        y.backward(dy)
        x.grad = w.grad = b.grad = None

    e = n * c * h * w_
    return run, {"fwd_bytes": 2 * e * 2, "bwd_bytes": 3 * e * 2}


def _geglu(rows, inner):
    x = torch.randn(rows, 2 * inner, device=DEV, dtype=BF, requires_grad=True)
    dy = torch.randn(rows, inner, device=DEV, dtype=BF)

    def run():
        y = ops.geglu(x)
        y.backward(dy)
        x.grad = None

    return run, {"fwd_bytes": 3 * rows * inner * 2, "bwd_bytes": 5 * rows * inner * 2}


def _xent(rows, vocab):
    logits = torch.randn(rows, vocab, device=DEV, dtype=BF, requires_grad=True)
    labels = torch.randint(0, vocab, (rows,), device=DEV)

    def run():
        loss = ops.cross_entropy(logits, labels, inplace_grad=False)
        loss.backward()
        logits.grad = None

    return run, {"fwd_bytes": rows * vocab * 2, "bwd_bytes": 2 * rows * vocab * 2}


def _adamw(n):
    from kubernetes_cloud_amd.train.optim import FlatAdamW

    master = torch.randn(n, device=DEV)
    bf = master.to(BF)
    opt = FlatAdamW(master, lr=1e-4, weight_decay=0.01, model_bf16=bf)
    opt.grad.normal_()

    def run():
        opt.step()

    # master rw, grad r, m rw, v rw, bf16 w
    return run, {"bytes": n * (4 * 2 + 4 + 4 * 2 + 4 * 2 + 2)}


def _gemv(n_out, k):
    from kubernetes_cloud_amd.ops.gemv import skinny_linear

    x = torch.randn(1, k, device=DEV, dtype=BF)
    w = torch.randn(n_out, k, device=DEV, dtype=BF) * 0.02
    b = torch.randn(n_out, device=DEV, dtype=BF)

    def run():
        skinny_linear(x, w, b, 1)

    return run, {"bytes": n_out * k * 2}


def _decode_attn(B, H, D, L):
    from kubernetes_cloud_amd.ops import decode as dops

    kc = torch.randn(B, H, L, D, device=DEV, dtype=BF)
    vc = torch.randn_like(kc)
    q = torch.randn(B, 3 * H * D, device=DEV, dtype=BF)
    slots = torch.arange(B, device=DEV, dtype=torch.int32)
    lens = torch.full((B,), L, device=DEV, dtype=torch.int32)

    def run():
        dops.decode_attention(q, kc, vc, slots, lens, H, L)

    return run, {"bytes": 2 * B * H * L * D * 2}


def _conv(N, H, W, C, Co):
    from kubernetes_cloud_amd.ops.conv import conv3x3

    x = torch.randn(N, C, H, W, device=DEV, dtype=BF).contiguous(memory_format=torch.channels_last)
    w = (torch.randn(Co, C, 3, 3, device=DEV, dtype=BF) * 0.02).contiguous(memory_format=torch.channels_last)

    def run():
        conv3x3(x, w)

    return run, {"flops": 2.0 * N * H * W * Co * 9 * C}


def _mm(M, N, K):
    from kubernetes_cloud_amd.ops import skinny_mm as smm

    x = torch.randn(M, K, device=DEV, dtype=BF)
    ws = [torch.randn(N, K, device=DEV, dtype=BF) * 0.02 for _ in range(4)]  # rotate: cold weights
    b = torch.randn(N, device=DEV, dtype=BF)
    it = [0]

    def run():
        smm.mm(x, ws[it[0] % 4], b)
        it[0] += 1

    return run, {"bytes": N * K * 2}


CASES = {
    "attn_gptj": lambda: _attn(8, 2048, 16, 256, True),
    "attn_sd64": lambda: _attn(16, 4096, 8, 40, False),
    "attn_sd_tiled48": lambda: _attn_sd_tiled(16, 4096, 8, 40, 48),
    "layernorm_gptj": lambda: _layernorm(16384, 4096),
    "groupnorm_nhwc_sd": lambda: _groupnorm(8, 320, 64, 64),
    "geglu_sd": lambda: _geglu(32768, 1280),
    "xent_gptj": lambda: _xent(16384, 50400),
    "adamw_512m": lambda: _adamw(512 * 1024 * 1024),
    "gemv_fcin_m1": lambda: _gemv(16384, 4096),
    "decode_attn_b32": lambda: _decode_attn(32, 16, 256, 2048),
    "conv_sd64": lambda: _conv(16, 64, 64, 320, 320),
    "mm_bloom_fcin_m8": lambda: _mm(8, 7168, 14336),
    "mm_bloom_fcout_m8": lambda: _mm(8, 14336, 7168),
    "conv_sd32": lambda: _conv(16, 32, 32, 640, 640),
}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--cases", default=",".join(CASES))
    ap.add_argument("--iters", type=int, default=3)
    ap.add_argument("--out", default="gpurun_out/pmc/cases.json")
    args = ap.parse_args()
    _lib.require()
    meta = {}
    for name in args.cases.split(","):
        run, model = CASES[name]()
        run()  # warm (first-call allocations, kernel loads)
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(args.iters):
            run()
        e.record()
        torch.cuda.synchronize()
        ms = s.elapsed_time(e) / args.iters
        meta[name] = dict(model, ms_per_iter=ms)
        print(f"[kernel_pmc] {name}: {ms:.3f} ms/iter", flush=True)
        del run
        torch.cuda.empty_cache()
    os.makedirs(os.path.dirname(args.out), exist_ok=True)
    with open(args.out, "w") as f:
        json.dump(meta, f, indent=1)


if __name__ == "__main__":
    main()
