"""LayerNorm (+ fused residual adds) and GroupNorm(+SiLU) autograd ops.

GPU tensors run ``csrc/kernels/layernorm.hip`` / ``groupnorm.hip``; CPU tensors
run the fp32 PyTorch reference below (the numerics the kernel tests compare
against).
"""
from __future__ import annotations

import torch
import torch.nn.functional as F

from . import _lib


def _ln_ref(h: torch.Tensor, w, b, eps):
    return F.layer_norm(h.float(), (h.shape[-1],), w.float() if w is not None else None,
                        b.float() if b is not None else None, eps).to(h.dtype)


class _LayerNormFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, bias, eps, r1, r2):
        d = x.shape[-1]
        rows = x.numel() // d
        x2 = x.contiguous()
        has_res = r1 is not None
        h = torch.empty_like(x2) if has_res else None
        y = torch.empty_like(x2)
        mean = torch.empty(rows, device=x.device, dtype=torch.float32)
        rstd = torch.empty(rows, device=x.device, dtype=torch.float32)
        # keep the contiguous copies alive until the launch: a temporary freed
        # inside the argument list is recycled by the next allocation (r2's copy)
        r1c = r1.contiguous() if r1 is not None else None
        r2c = r2.contiguous() if r2 is not None else None
        _lib.call("kca_layernorm_fwd", x2.data_ptr(), _lib.ptr(r1c), _lib.ptr(r2c), _lib.ptr(h),
                  weight.data_ptr(), _lib.ptr(bias), y.data_ptr(), mean.data_ptr(),
                  rstd.data_ptr(), rows, d, float(eps), _lib.stream())
        ctx.save_for_backward(h if has_res else x2, weight, mean, rstd)
        ctx.has_bias = bias is not None
        ctx.has_res = has_res
        ctx.n_res = (r1 is not None) + (r2 is not None)
        if has_res:
            return y, h
        return y, None

    @staticmethod
    def backward(ctx, dy, dh):
        h, weight, mean, rstd = ctx.saved_tensors
        d = h.shape[-1]
        rows = h.numel() // d
        dy = dy.contiguous()
        dx = torch.empty_like(h)
        parts = _lib.require().kca_layernorm_bwd_parts(rows)
        ws = torch.empty(2 * parts * d, device=h.device, dtype=torch.float32)
        dw = torch.empty_like(weight)
        db = torch.empty_like(weight) if ctx.has_bias else None
        dres = dh.contiguous() if (ctx.has_res and dh is not None) else None
        _lib.call("kca_layernorm_bwd", dy.data_ptr(), h.data_ptr(), mean.data_ptr(),
                  rstd.data_ptr(), weight.data_ptr(), _lib.ptr(dres), dx.data_ptr(),
                  dw.data_ptr(), _lib.ptr(db), int(weight.dtype == torch.float32),
                  ws.data_ptr(), rows, d, _lib.stream())
        g1 = dx if ctx.n_res >= 1 else None
        g2 = dx if ctx.n_res >= 2 else None
        return dx, dw, db, None, g1, g2


def layer_norm(x: torch.Tensor, weight: torch.Tensor, bias: torch.Tensor | None,
               eps: float = 1e-5, residual: tuple = ()):
    """LayerNorm over the last dim, optionally of ``x + sum(residual)``.

    Returns ``y`` when ``residual`` is empty, else ``(y, h)`` with
    ``h = x + sum(residual)`` (the new residual stream, stored once).
    """
    r1 = residual[0] if len(residual) > 0 else None
    r2 = residual[1] if len(residual) > 1 else None
    if len(residual) > 2:
        raise ValueError("at most two fused residual adds")
    if _lib.use_native(x):
        y, h = _LayerNormFn.apply(x, weight, bias, eps, r1, r2)
        return (y, h) if residual else y
    h = x
    for r in residual:
        h = h + r
    y = _ln_ref(h, weight, bias, eps)
    return (y, h) if residual else y


# ------------------------------------------------------------------ GroupNorm
class _GroupNormFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, bias, groups, eps, silu):
        # x: [N, C, *spatial] contiguous (NCHW) bf16
        x = x.contiguous()
        n, c = x.shape[0], x.shape[1]
        hw = x.numel() // (n * c)
        y = torch.empty_like(x)
        mean = torch.empty(n * groups, device=x.device, dtype=torch.float32)
        rstd = torch.empty_like(mean)
        part = torch.empty(2 * n * c, device=x.device, dtype=torch.float32)
        _lib.call("kca_groupnorm_fwd", x.data_ptr(), weight.data_ptr(), _lib.ptr(bias),
                  y.data_ptr(), mean.data_ptr(), rstd.data_ptr(), part.data_ptr(), n, c, hw, groups,
                  float(eps), int(silu), _lib.stream())
        ctx.save_for_backward(x, weight, bias, mean, rstd)
        ctx.groups, ctx.silu = groups, silu
        return y

    @staticmethod
    def backward(ctx, dy):
        x, weight, bias, mean, rstd = ctx.saved_tensors
        n, c = x.shape[0], x.shape[1]
        hw = x.numel() // (n * c)
        dy = dy.contiguous()
        dx = torch.empty_like(x)
        dw = torch.empty_like(weight)
        db = torch.empty_like(weight)
        ws = torch.empty(4 * n * c, device=x.device, dtype=torch.float32)
        _lib.call("kca_groupnorm_bwd", dy.data_ptr(), x.data_ptr(), weight.data_ptr(),
                  _lib.ptr(bias), mean.data_ptr(), rstd.data_ptr(), dx.data_ptr(),
                  dw.data_ptr(), db.data_ptr(), ws.data_ptr(), n, c, hw, ctx.groups,
                  int(ctx.silu), _lib.stream())
        return dx, dw, (db if bias is not None else None), None, None, None


class _GroupNormNHWCFn(torch.autograd.Function):
    """Channels-last [N, C, H, W] (memory NHWC): csrc/kernels/groupnorm_nhwc.hip."""

    @staticmethod
    def forward(ctx, x, weight, bias, groups, eps, silu):
        n, c = x.shape[0], x.shape[1]
        p = x.numel() // (n * c)
        y = torch.empty_like(x)
        mean = torch.empty(n * groups, device=x.device, dtype=torch.float32)
        rstd = torch.empty_like(mean)
        ws = torch.empty(_lib.require().kca_groupnorm_nhwc_ws(n, p, c), device=x.device, dtype=torch.float32)
        _lib.call("kca_groupnorm_nhwc_fwd", x.data_ptr(), weight.data_ptr(), _lib.ptr(bias), y.data_ptr(),
                  mean.data_ptr(), rstd.data_ptr(), ws.data_ptr(), n, p, c, groups, float(eps), int(silu),
                  _lib.stream())
        ctx.save_for_backward(x, weight, bias, mean, rstd)
        ctx.groups, ctx.silu = groups, silu
        return y

    @staticmethod
    def backward(ctx, dy):
        x, weight, bias, mean, rstd = ctx.saved_tensors
        n, c = x.shape[0], x.shape[1]
        p = x.numel() // (n * c)
        dy = dy.contiguous(memory_format=torch.channels_last)
        dx = torch.empty_like(x)
        dw = torch.empty_like(weight)
        db = torch.empty_like(weight) if bias is not None else None
        ws = torch.empty(_lib.require().kca_groupnorm_nhwc_ws(n, p, c) + 2 * n * ctx.groups, device=x.device,
                         dtype=torch.float32)
        _lib.call("kca_groupnorm_nhwc_bwd", dy.data_ptr(), x.data_ptr(), weight.data_ptr(), _lib.ptr(bias),
                  mean.data_ptr(), rstd.data_ptr(), dx.data_ptr(), dw.data_ptr(), _lib.ptr(db), ws.data_ptr(),
                  n, p, c, ctx.groups, int(ctx.silu), _lib.stream())
        return dx, dw, db, None, None, None


def _channels_last(x: torch.Tensor) -> bool:
    return x.dim() == 4 and x.is_contiguous(memory_format=torch.channels_last) and not x.is_contiguous()


def _group_norm_nhwc_add(x, add, weight, bias, groups, eps, silu):
    """Inference GroupNorm of ``x + add[:, :, None, None]`` without forming the sum."""
    n, c = x.shape[0], x.shape[1]
    p = x.numel() // (n * c)
    add = add.to(torch.float32)
    if add.stride(1) != 1 or add.stride(0) < c:  # a row-strided slice (the UNet's batched time GEMM) is read in place
        add = add.contiguous()
    y = torch.empty_like(x)
    mean = torch.empty(n * groups, device=x.device, dtype=torch.float32)
    rstd = torch.empty_like(mean)
    ws = torch.empty(_lib.require().kca_groupnorm_nhwc_ws(n, p, c), device=x.device, dtype=torch.float32)
    _lib.call("kca_groupnorm_nhwc_fwd_add", x.data_ptr(), weight.data_ptr(), _lib.ptr(bias), add.data_ptr(),
              add.stride(0), y.data_ptr(), mean.data_ptr(), rstd.data_ptr(), ws.data_ptr(), n, p, c, groups, float(eps),
              int(silu), _lib.stream())
    return y


def phase_to_dense(ph: torch.Tensor, hw: tuple) -> torch.Tensor:
    """The upsampler's sub-pixel phase layout -> the dense upsampled tensor (reference / fallback):
    ph [N, 4C, H/2+1, W/2+1] holds output phase (a, b) in channel block 2a + b at offset (a, b)."""
    H, W = hw
    C = ph.shape[1] // 4
    out = ph.new_empty(ph.shape[0], C, H, W)
    for a in range(2):
        for b in range(2):
            k = 2 * a + b
            out[:, :, a::2, b::2] = ph[:, k * C:(k + 1) * C, a:a + H // 2, b:b + W // 2]
    return out


def group_norm_cat(x1: torch.Tensor, x2: torch.Tensor, groups: int, weight: torch.Tensor,
                   bias: torch.Tensor | None, eps: float = 1e-5, silu: bool = False, phase: bool = False,
                   x1_add: torch.Tensor | None = None, want_raw: bool = True):
    """Inference GroupNorm(+SiLU) of the channel concat ``[x1 + x1_add | x2]`` without a
    concatenated copy for the norm (``kca_groupnorm_nhwc_cat_fwd``): returns ``(y, raw)`` with
    ``raw`` the concat itself (None unless ``want_raw``), both channels-last [N, C1 + C2, H, W].
    ``phase``: x1 is still in the upsampler's phase layout (``phase_to_dense``); ``x1_add``: a
    per-channel [C1] vector (the upsampler conv's bias) added to x1."""
    N, C2, H, W = x2.shape
    C1 = x1.shape[1] // (4 if phase else 1)
    native = (_lib.use_native(x1, x2) and not torch.is_grad_enabled() and x1.dtype == torch.bfloat16
              and x2.dtype == torch.bfloat16 and _channels_last(x1) and _channels_last(x2) and C1 % 8 == 0
              and C2 % 8 == 0 and weight is not None and _lib.has("kca_groupnorm_nhwc_cat_fwd")
              and (not phase or (H % 2 == 0 and W % 2 == 0 and tuple(x1.shape[2:]) == (H // 2 + 1, W // 2 + 1))))
    if not native:
        d1 = phase_to_dense(x1, (H, W)) if phase else x1
        if x1_add is not None:
            d1 = d1 + x1_add.to(d1.dtype)[None, :, None, None]
        cat = torch.cat([d1, x2], dim=1)
        return group_norm(cat, groups, weight, bias, eps, silu=silu), (cat if want_raw else None)
    C, P = C1 + C2, H * W
    y = torch.empty(N, H, W, C, device=x2.device, dtype=x2.dtype).permute(0, 3, 1, 2)
    raw = torch.empty(N, H, W, C, device=x2.device, dtype=x2.dtype).permute(0, 3, 1, 2) if want_raw else None
    add = None
    if x1_add is not None:
        add = torch.zeros(N, C, device=x2.device, dtype=torch.float32)
        add[:, :C1] = x1_add.float()
    mean = torch.empty(N * groups, device=x2.device, dtype=torch.float32)
    rstd = torch.empty_like(mean)
    ws = torch.empty(_lib.require().kca_groupnorm_nhwc_ws(N, P, C), device=x2.device, dtype=torch.float32)
    _lib.call("kca_groupnorm_nhwc_cat_fwd", x1.data_ptr(), x2.data_ptr(), weight.data_ptr(), _lib.ptr(bias),
              _lib.ptr(add), y.data_ptr(), _lib.ptr(raw), mean.data_ptr(), rstd.data_ptr(), ws.data_ptr(), N, P, C1,
              C2, W if phase else 0, groups, float(eps), int(silu), _lib.stream())
    return y, raw


def group_norm(x: torch.Tensor, groups: int, weight: torch.Tensor, bias: torch.Tensor | None,
               eps: float = 1e-5, silu: bool = False, add: torch.Tensor | None = None) -> torch.Tensor:
    """GroupNorm over NC* tensors, optionally fused with SiLU (UNet/VAE ResNet blocks).
    Channels-last 4-D inputs stay channels-last (NHWC kernels). ``add`` ([N, C]):
    normalise ``x + add[:, :, None, None]`` (the ResNet block's time embedding);
    fused into the statistics and the apply pass when no gradient is needed."""
    nhwc = (_lib.use_native(x) and x.dtype == torch.bfloat16 and _channels_last(x) and x.shape[1] % 8 == 0
            and weight is not None and _lib.has("kca_groupnorm_nhwc_fwd"))
    if add is not None:
        if (nhwc and not torch.is_grad_enabled() and add.shape == x.shape[:2]
                and _lib.has("kca_groupnorm_nhwc_fwd_add")):
            return _group_norm_nhwc_add(x, add, weight, bias, groups, eps, silu)
        x = x + add[:, :, None, None]
    if nhwc:
        return _GroupNormNHWCFn.apply(x, weight, bias, groups, eps, silu)
    if _lib.use_native(x) and x.dtype == torch.bfloat16 and _lib.has("kca_groupnorm_fwd"):
        return _GroupNormFn.apply(x, weight, bias, groups, eps, silu)
    if _lib.use_native(x) and x.dtype == torch.bfloat16:
        _lib.require()
        raise RuntimeError("kca_groupnorm_fwd missing from the kernel library")
    y = F.group_norm(x.float(), groups, weight.float() if weight is not None else None,
                     bias.float() if bias is not None else None, eps)
    if silu:
        y = F.silu(y)
    return y.to(x.dtype)
