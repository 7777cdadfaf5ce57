#!/usr/bin/env python3
"""SD-1.5 UNet upsamplers: nearest x2 + 3x3 conv, against the sub-pixel form that convolves the
low-resolution input with the four 2x2 phase kernels (one 2x2 conv, 4*C outputs, padding 1).

    python bench/upsample_conv_bench.py

Nearest-x2 followed by a 3x3 conv touches each input pixel through 2x2 distinct weight sums per
output phase, so the phase form does 16 instead of 36 multiply-adds per (input pixel, Cin, Cout)
and never materialises the 4x upsampled activation. One JSON line per shape (CFG batch 16,
channels-last bf16, MIOpen): ms for upsample+conv3x3, conv3x3 alone, the 2x2 phase conv through
MIOpen, and the framework's path (ops/upsample.py: im2col + one hipBLASLt GEMM, phase layout out;
``phase_gemm_dense_ms`` adds the densifying scatter + bias the VAE decoder needs).
"""
from __future__ import annotations

import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch
import torch.nn.functional as F

SHAPES = [(16, 1280, 8), (16, 1280, 16), (16, 640, 32)]  # (batch, channels, low-res side)


def _time(fn, iters=20, warmup=5):
    for _ in range(warmup):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters


def main():
    from kubernetes_cloud_amd.ops.upsample import (phase_gemm_weights, phase_to_dense, phase_weights,
                                                   upsample_conv_phase)
    from kubernetes_cloud_amd.utils import miopen
    miopen.configure()
    dev = "cuda"
    cl = torch.channels_last
    for B, C, S in SHAPES:
        x = torch.randn(B, C, S, S, device=dev, dtype=torch.bfloat16).contiguous(memory_format=cl)
        w = (torch.randn(C, C, 3, 3, device=dev) * (9 * C) ** -0.5).bfloat16().contiguous(memory_format=cl)
        wp = phase_weights(w).contiguous(memory_format=cl)
        with torch.no_grad():
            up = F.interpolate(x, scale_factor=2.0, mode="nearest")
            t_up = _time(lambda: F.conv2d(F.interpolate(x, scale_factor=2.0, mode="nearest"), w, padding=1))
            t_conv = _time(lambda: F.conv2d(up, w, padding=1))
            t_ph = _time(lambda: F.conv2d(x, wp, padding=1))
            wg = phase_gemm_weights(w)
            t_gemm = _time(lambda: upsample_conv_phase(x, wg))
            t_gemm_d = _time(lambda: phase_to_dense(upsample_conv_phase(x, wg), (2 * S, 2 * S)))
            gd = phase_to_dense(upsample_conv_phase(x, wg), (2 * S, 2 * S)).float()
            gerr = ((gd - F.conv2d(up.float(), w.float(), padding=1)).abs().max()).item()
            ref = F.conv2d(up.float(), w.float(), padding=1)
            ph = F.conv2d(x, wp, padding=1).float()
            out = torch.empty_like(ref)
            for a in range(2):
                for b in range(2):
                    k = 2 * a + b
                    out[:, :, a::2, b::2] = ph[:, k * C:(k + 1) * C, a:a + S, b:b + S]
            err = ((out - ref).abs().max() / ref.abs().max()).item()
        print(json.dumps({"B": B, "C": C, "low_res": S, "upsample_conv3x3_ms": round(t_up, 4),
                          "conv3x3_only_ms": round(t_conv, 4), "phase_conv2x2_ms": round(t_ph, 4),
                          "phase_gemm_ms": round(t_gemm, 4), "phase_gemm_dense_ms": round(t_gemm_d, 4),
                          "phase_rel_err": round(err, 5), "phase_gemm_abs_err": round(gerr, 5)}), flush=True)


if __name__ == "__main__":
    main()
