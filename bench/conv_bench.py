#!/usr/bin/env python3
"""SD-1.5 UNet 3x3 convolutions (channels-last bf16, txt2img batch 8 + CFG = 16) on MI355X:
MIOpen (tuned db, utils/miopen.py) vs the matrix-core implicit GEMM (ops/conv.py) (and, with
KCA_CONV_BENCH_IM2COL=1, an explicit NHWC im2col + hipBLASLt GEMM).

    python bench/conv_bench.py
"""
from __future__ import annotations

import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch
import torch.nn.functional as F

from kubernetes_cloud_amd.utils import miopen

# (N, H, W, Cin, Cout)
SHAPES = [(16, 64, 64, 320, 320), (16, 64, 64, 640, 320), (16, 32, 32, 320, 640), (16, 32, 32, 640, 640),
          (16, 16, 16, 640, 1280), (16, 16, 16, 1280, 1280), (16, 8, 8, 1280, 1280), (16, 8, 8, 2560, 1280),
          (16, 16, 16, 2560, 1280), (16, 32, 32, 1280, 640), (16, 64, 64, 960, 320),
          # the VAE decoder at the txt2img batch (8)
          (8, 64, 64, 512, 512), (8, 128, 128, 512, 512), (8, 256, 256, 512, 256), (8, 256, 256, 256, 256),
          (8, 512, 512, 256, 128), (8, 512, 512, 128, 128)]


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


def im2col_conv(x, w2):
    """x [N, C, H, W] channels-last, w2 [Cout, 9*C] (kh, kw, C order) -> y [N, Cout, H, W] channels-last."""
    N, C, H, W = x.shape
    xp = F.pad(x, (1, 1, 1, 1))  # stays channels-last
    xn = xp.permute(0, 2, 3, 1)   # [N, H+2, W+2, C] view
    sN, sH, sW, sC = xn.stride()
    cols = xn.as_strided((N, H, W, 3, 3, C), (sN, sH, sW, sH, sW, sC)).reshape(N * H * W, 9 * C)
    y = cols @ w2.t()
    return y.view(N, H, W, -1).permute(0, 3, 1, 2)


def main():
    miopen.configure()
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    for (N, H, W, Ci, Co) in SHAPES:
        x = torch.randn(N, Ci, H, W, device=dev, dtype=torch.bfloat16).to(memory_format=torch.channels_last)
        w = (torch.randn(Co, Ci, 3, 3, device=dev, dtype=torch.bfloat16) * 0.02).to(memory_format=torch.channels_last)
        w2 = w.permute(0, 2, 3, 1).reshape(Co, 9 * Ci).contiguous()
        flops = 2.0 * N * H * W * Co * 9 * Ci
        t_conv = timeit(lambda: F.conv2d(x, w, padding=1))
        from kubernetes_cloud_amd.ops import conv as kconv
        from kubernetes_cloud_amd.ops.conv import supported
        kconv._MODE = "all"  # the kernel on every supported shape (the model dispatch uses kconv._FAST)
        conv3x3 = kconv.conv3x3
        rec = {"shape": [N, H, W, Ci, Co], "miopen_ms": round(t_conv, 4), "miopen_tflops": round(flops / t_conv / 1e9, 1)}
        if supported(x, w):
            t_ig = timeit(lambda: conv3x3(x, w))
            ref = F.conv2d(x.float(), w.float(), padding=1)
            err = float((ref - conv3x3(x, w).float()).abs().max() / (ref.abs().max() + 1e-6))
            rec.update(igemm_ms=round(t_ig, 4), igemm_tflops=round(flops / t_ig / 1e9, 1), igemm_rel_err=round(err, 5))
        if os.environ.get("KCA_CONV_BENCH_IM2COL"):
            t_col = timeit(lambda: im2col_conv(x, w2))
            rec.update(im2col_gemm_ms=round(t_col, 4), im2col_tflops=round(flops / t_col / 1e9, 1))
        print(json.dumps(rec), flush=True)

if __name__ == "__main__":
    main()
