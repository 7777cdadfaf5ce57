"""Activation ops: tanh-GELU (GPT-J/NeoX/BLOOM/GPT-2 "gelu_new") and GEGLU."""
from __future__ import annotations

import torch
import torch.nn.functional as F

from . import _lib


class _GeluFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, u, approx):
        u = u.contiguous()
        y = torch.empty_like(u)
        _lib.call("kca_gelu_fwd", u.data_ptr(), y.data_ptr(), u.numel(), int(approx), _lib.stream())
        ctx.save_for_backward(u)
        ctx.approx = approx
        return y

    @staticmethod
    def backward(ctx, dy):
        (u,) = ctx.saved_tensors
        du = torch.empty_like(u)
        dy = dy.contiguous()
        _lib.call("kca_gelu_bwd", dy.data_ptr(), u.data_ptr(), du.data_ptr(),
                  u.numel(), int(ctx.approx), _lib.stream())
        return du, None


def gelu(u: torch.Tensor, approximate: str = "tanh") -> torch.Tensor:
    """GELU of the pre-activation ``u`` (bias already added by the GEMM
    epilogue); ``approximate`` is "tanh" (gelu_new / gelu_fast) or "none" (erf)."""
    approx = approximate == "tanh"
    if _lib.use_native(u) and u.numel() % 8 == 0:
        return _GeluFn.apply(u, approx)
    return F.gelu(u.float(), approximate="tanh" if approx else "none").to(u.dtype)


class _QuickGeluFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, u):
        u = u.contiguous()
        y = torch.empty_like(u)
        _lib.call("kca_quick_gelu_fwd", u.data_ptr(), y.data_ptr(), u.numel(), _lib.stream())
        ctx.save_for_backward(u)
        return y

    @staticmethod
    def backward(ctx, dy):
        (u,) = ctx.saved_tensors
        dy = dy.contiguous()
        du = torch.empty_like(u)
        _lib.call("kca_quick_gelu_bwd", dy.data_ptr(), u.data_ptr(), du.data_ptr(), u.numel(), _lib.stream())
        return du


def quick_gelu(x: torch.Tensor) -> torch.Tensor:
    """CLIP's x * sigmoid(1.702 x): one native pass on bf16 GPU tensors (torch: mul + sigmoid + mul)."""
    if _lib.use_native(x) and x.numel() % 8 == 0:
        return _QuickGeluFn.apply(x)
    return x * torch.sigmoid(1.702 * x)


class _GegluFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x):
        x = x.contiguous()
        inner = x.shape[-1] // 2
        rows = x.numel() // x.shape[-1]
        y = torch.empty(*x.shape[:-1], inner, device=x.device, dtype=x.dtype)
        _lib.call("kca_geglu_fwd", x.data_ptr(), y.data_ptr(), rows, inner, _lib.stream())
        ctx.save_for_backward(x)
        return y

    @staticmethod
    def backward(ctx, dy):
        (x,) = ctx.saved_tensors
        dy = dy.contiguous()
        dx = torch.empty_like(x)
        _lib.call("kca_geglu_bwd", dy.data_ptr(), x.data_ptr(), dx.data_ptr(), x.numel() // x.shape[-1],
                  x.shape[-1] // 2, _lib.stream())
        return dx


def geglu(x: torch.Tensor) -> torch.Tensor:
    """diffusers GEGLU: split the projection in half, value * gelu(gate) (exact erf).
    GPU: one fused pass (kca_geglu_fwd / _bwd)."""
    if _lib.use_native(x) and (x.shape[-1] // 2) % 8 == 0 and x.shape[-1] % 2 == 0:
        return _GegluFn.apply(x)
    a, g = x.chunk(2, dim=-1)
    return a * F.gelu(g.float()).to(a.dtype)


def add_bias_nhwc(a: torch.Tensor, b: torch.Tensor | None, bias: torch.Tensor) -> torch.Tensor:
    """``a + b + bias[None, :, None, None]`` for channels-last [N, C, H, W] bf16 tensors in one
    pass (``kca_add_bias_nhwc``): the SD ResNet block's residual add with the convolution biases
    folded in (models/unet.py). Inference helper: no autograd."""
    ok = (_lib.use_native(a) and a.dtype == torch.bfloat16 and a.dim() == 4 and a.shape[1] % 8 == 0
          and a.is_contiguous(memory_format=torch.channels_last)
          and (b is None or (b.shape == a.shape and b.dtype == a.dtype
                             and b.is_contiguous(memory_format=torch.channels_last))))
    if not ok:
        y = a.float() + (b.float() if b is not None else 0.0) + bias.float()[None, :, None, None]
        return y.to(a.dtype)
    out = torch.empty_like(a)
    bf = bias.float().contiguous()
    _lib.call("kca_add_bias_nhwc", a.data_ptr(), _lib.ptr(b), bf.data_ptr(), out.data_ptr(), a.numel(),
              a.shape[1], _lib.stream())
    return out


class _AddBiasNHWCFn(torch.autograd.Function):
    """Training form of ``add_bias_nhwc``: forward in one native pass; backward hands ``dout`` to
    both summands and the bias gradient is the column sum of ``dout`` viewed as [N*H*W, C]
    (``ops.linear.column_sum``) -- instead of a separate biased convolution's broadcast add and
    PyTorch's reduction over the full activation."""

    @staticmethod
    def forward(ctx, a, b, bias):
        ctx.C = a.shape[1]
        ctx.has_b = b is not None
        return add_bias_nhwc(a, b, bias)

    @staticmethod
    def backward(ctx, dout):
        from .linear import column_sum
        d = dout.contiguous(memory_format=torch.channels_last)
        db = column_sum(d.permute(0, 2, 3, 1).reshape(-1, ctx.C), out_dtype=torch.float32)
        return d, (d if ctx.has_b else None), db


class _AddBias2NHWCFn(torch.autograd.Function):
    """``a + b + bias1 + bias2`` (channels-last) with the bf16 bias parameters read in the kernel; the
    backward's column sum lands in bf16 once and is the gradient of both biases."""

    @staticmethod
    def forward(ctx, a, b, bias1, bias2):
        ctx.C = a.shape[1]
        ctx.has_b, ctx.has_b2 = b is not None, bias2 is not None
        out = torch.empty_like(a)
        _lib.call("kca_add_bias2_nhwc", a.data_ptr(), _lib.ptr(b), bias1.data_ptr(), _lib.ptr(bias2),
                  out.data_ptr(), a.numel(), a.shape[1], _lib.stream())
        return out

    @staticmethod
    def backward(ctx, dout):
        from .linear import column_sum
        d = dout.contiguous(memory_format=torch.channels_last)
        db = column_sum(d.permute(0, 2, 3, 1).reshape(-1, ctx.C), out_dtype=torch.bfloat16)
        return d, (d if ctx.has_b else None), db, (db if ctx.has_b2 else None)


def add_bias2_nhwc_train(a: torch.Tensor, b: torch.Tensor | None, bias1: torch.Tensor,
                         bias2: torch.Tensor | None) -> torch.Tensor:
    """``a + b + bias1 + bias2`` for the SD ResNet block's residual add (training): bf16 biases as
    parameters, one native pass; falls back to add_bias_nhwc_train off the fast path."""
    ok = (_lib.use_native(a, bias1) and a.dim() == 4 and a.shape[1] % 8 == 0 and bias1.is_contiguous()
          and a.is_contiguous(memory_format=torch.channels_last) and _lib.has("kca_add_bias2_nhwc")
          and (bias2 is None or (bias2.dtype == torch.bfloat16 and bias2.is_contiguous()))
          and (b is None or (b.shape == a.shape and b.dtype == a.dtype
                             and b.is_contiguous(memory_format=torch.channels_last))))
    if not ok:
        bias = bias1.float() + (bias2.float() if bias2 is not None else 0.0)
        return add_bias_nhwc_train(a, b, bias)
    return _AddBias2NHWCFn.apply(a, b, bias1, bias2)


def add_bias_nhwc_train(a: torch.Tensor, b: torch.Tensor | None, bias: torch.Tensor) -> torch.Tensor:
    """``a + b + bias`` (channels-last) with autograd; the inference kernel when no grad is recorded."""
    if torch.is_grad_enabled() and (a.requires_grad or (b is not None and b.requires_grad) or bias.requires_grad):
        return _AddBiasNHWCFn.apply(a, b, bias)
    return add_bias_nhwc(a, b, bias)
