"""3x3 convolution on the matrix cores (``csrc/kernels/conv_igemm.hip``: implicit GEMM over NHWC, no im2col
buffer) for the SD-1.5 UNet / VAE convolutions.

``conv3x3(x, w, bias)`` takes channels-last bf16 tensors (the layout the SD models run in,
``models/unet.py`` ``to_channels_last``): x [N, C, H, W], w [Cout, C, 3, 3] (physically NHWC / KRSC),
stride 1, padding 1. Shapes the kernel does not take (C or Cout not a multiple of 64, N*H*W not a
multiple of 128, other dtypes / layouts, CPU tensors) run ``F.conv2d``. Forward only: under autograd
the backward is PyTorch's ``convolution_backward`` (MIOpen).
"""
from __future__ import annotations

import os

import torch
import torch.nn.functional as F

from . import _lib

# "1" (default): the measured shapes below, "all": every supported shape, "0": off (MIOpen everywhere).
# End to end on the same box, KCA_CONV_IGEMM=0 -> 1: txt2img 6.378 / 6.416 -> 6.498 / 6.537 images/s,
# DreamBooth 61.99 / 61.93 -> 62.16 / 62.31 samples/s (profiles/conv_sd_ab_r6.jsonl)
_MODE = os.environ.get("KCA_CONV_IGEMM", "1")
# (H, W, C, Cout) where the kernel (LDS-DMA form) beat the tuned MIOpen solvers in same-box runs
# (profiles/conv_bench_r6.jsonl; UNet at N = 16, VAE decoder at N = 8): UNet 64x64 640 / 960 -> 320 773 /
# 799 vs 625 / 704 TFLOP/s, 320 -> 320 684 vs 642, the 16x16 convs 606-686 vs 524-530; the VAE's 512x512
# convs 871 / 792 vs 766 / 718. MIOpen keeps the UNet's 32x32 convs (606-663 vs 729-784: 320 workgroups
# are 1.25 rounds of the chip), its 8x8 ones (16 blocks) and the VAE's 64-256 px convs (~1 PF there).
_FAST = {(64, 64, 320, 320), (64, 64, 640, 320), (64, 64, 960, 320), (16, 16, 640, 1280), (16, 16, 1280, 1280),
         (16, 16, 2560, 1280), (16, 16, 1920, 1280), (512, 512, 256, 128), (512, 512, 128, 128)}
_VARIANT_SET = False


def supported(x: torch.Tensor, w: torch.Tensor) -> bool:
    if not (x.is_cuda and x.dtype == torch.bfloat16 and w.dtype == torch.bfloat16 and x.dim() == 4
            and w.dim() == 4 and tuple(w.shape[2:]) == (3, 3)):
        return False
    N, C, H, W = x.shape
    Co = w.shape[0]
    return (w.shape[1] == C and C % 64 == 0 and Co % 64 == 0 and (N * H * W) % 128 == 0
            and x.is_contiguous(memory_format=torch.channels_last)
            and w.is_contiguous(memory_format=torch.channels_last)
            and x.data_ptr() % 16 == 0 and w.data_ptr() % 16 == 0 and _lib.has("kca_conv3x3_fwd"))


def _fwd(x, w, bias):
    global _VARIANT_SET
    if not _VARIANT_SET:  # A/B: 1 = 128 x 128 tiles, 2 = 256 x 128 tiles (0: by shape)
        _VARIANT_SET = True
        v = int(os.environ.get("KCA_CONV_VARIANT", "0"))
        if v:
            _lib.call("kca_conv3x3_set_variant", v)
    N, C, H, W = x.shape
    Co = w.shape[0]
    y = torch.empty((N, Co, H, W), device=x.device, dtype=x.dtype, memory_format=torch.channels_last)
    b = bias if bias is not None and bias.dtype == x.dtype and bias.is_contiguous() else None
    _lib.call("kca_conv3x3_fwd", x.data_ptr(), w.data_ptr(), _lib.ptr(b), y.data_ptr(), N, H, W, C, Co,
              _lib.stream())
    if bias is not None and b is None:
        y = y + bias.view(1, -1, 1, 1)
    return y


class _Conv3x3(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, bias):
        ctx.save_for_backward(x, w)
        ctx.has_bias = bias is not None
        return _fwd(x, w, bias)

    @staticmethod
    def backward(ctx, gy):
        x, w = ctx.saved_tensors
        gx, gw, gb = torch.ops.aten.convolution_backward(
            gy.contiguous(memory_format=torch.channels_last), x, w, [w.shape[0]] if ctx.has_bias else None,
            [1, 1], [1, 1], [1, 1], False, [0, 0], 1,
            [ctx.needs_input_grad[0], ctx.needs_input_grad[1], ctx.has_bias and ctx.needs_input_grad[2]])
        return gx, gw, gb


def conv3x3(x: torch.Tensor, w: torch.Tensor, bias: torch.Tensor | None = None) -> torch.Tensor:
    """stride 1, padding 1 3x3 convolution (see module docstring)."""
    if _MODE in ("0", "false") or not supported(x, w) or \
            (_MODE != "all" and (x.shape[2], x.shape[3], x.shape[1], w.shape[0]) not in _FAST):
        return F.conv2d(x, w, bias, padding=1)
    if torch.is_grad_enabled() and (x.requires_grad or w.requires_grad or (bias is not None and bias.requires_grad)):
        return _Conv3x3.apply(x, w, bias)
    return _fwd(x, w, bias)


def conv3x3_reference(x, w, bias=None):
    """fp32 reference of ``conv3x3``."""
    return F.conv2d(x.float(), w.float(), bias.float() if bias is not None else None, padding=1)
