"""SD-1.5 upsamplers (nearest x2 + 3x3 conv) as one GEMM: csrc/kernels/sd_upsample.hip.

The UNet's three and the VAE decoder's three upsamplers
(online-inference/stable-diffusion/service/service.py:244-252 runs both per image) are
``conv3x3(nearest_x2(x))``. Per output phase (a, b) that is a 2x2 conv of the low-resolution input
(``phase_weights``): 16 instead of 36 multiply-adds per (input pixel, Cin, Cout), and no 4x
upsampled activation. ``upsample_conv_phase`` runs it as im2col (one bandwidth pass) + one
hipBLASLt GEMM whose output is the *phase layout* [N, h+1, w+1, 4C]: the UNet's concat GroupNorm
reads it in place (ops.norms.group_norm_cat ``phase=True``); ``phase_to_dense`` materialises it
(+ the conv bias) for the VAE decoder.
"""
from __future__ import annotations

import torch
import torch.nn.functional as F

from . import _lib

# nearest-x2 then 3x3 conv (padding 1) == per output phase (a, b) a 2x2 conv of the low-resolution
# input (padding 1, output window offset (a, b)) whose taps sum the 3x3 taps that land on the same
# input pixel: rows/cols {0} {1,2} for phase 0 and {0,1} {2} for phase 1
_PHASE_TAPS = (((0,), (1, 2)), ((0, 1), (2,)))


def _tap_matrix(device) -> torch.Tensor:
    """M[a, s, u] = 1 when 3x3 tap row u lands on input row s of output phase a (_PHASE_TAPS)."""
    m = torch.zeros(2, 2, 3, device=device)
    for a in range(2):
        for s_ in range(2):
            for u in _PHASE_TAPS[a][s_]:
                m[a, s_, u] = 1.0
    return m


def phase_weights(w: torch.Tensor) -> torch.Tensor:
    """[Cout, Cin, 3, 3] -> [4 * Cout, Cin, 2, 2]: output channel block k = 2a + b holds phase (a, b).
    One einsum with the 0/1 tap matrix (fp32), so the training backward is one einsum too."""
    m = _tap_matrix(w.device)
    out = torch.einsum("asu,btv,oiuv->aboist", m, m, w.float())
    return out.reshape(4 * w.shape[0], w.shape[1], 2, 2).to(w.dtype)


def phase_gemm_weights(w: torch.Tensor) -> torch.Tensor:
    """[Cout, Cin, 3, 3] -> the GEMM operand [4 * Cout, 4 * Cin], K in im2col order (s, t, cin)."""
    wp = phase_weights(w)
    return wp.permute(0, 2, 3, 1).reshape(wp.shape[0], 4 * w.shape[1]).contiguous()


def _nhwc(x: torch.Tensor) -> bool:
    return x.dim() == 4 and x.is_contiguous(memory_format=torch.channels_last)


def native_ok(x: torch.Tensor) -> bool:
    return (_lib.use_native(x) and _nhwc(x) and x.shape[1] % 8 == 0 and x.data_ptr() % 16 == 0
            and _lib.has("kca_im2col2x2_nhwc"))


def im2col2x2(x: torch.Tensor) -> torch.Tensor:
    """x [N, C, h, w] channels-last -> [N*(h+1)*(w+1), 4C]: the 2x2 (padding 1) patches, (s, t, c)."""
    N, C, h, w = x.shape
    if native_ok(x):
        a = torch.empty(N * (h + 1) * (w + 1), 4 * C, device=x.device, dtype=x.dtype)
        _lib.call("kca_im2col2x2_nhwc", x.data_ptr(), a.data_ptr(), N, h, w, C, _lib.stream())
        return a
    xp = F.pad(x.permute(0, 2, 3, 1), (0, 0, 1, 1, 1, 1))  # [N, h+2, w+2, C]
    taps = [xp[:, s:s + h + 1, t:t + w + 1, :] for s in range(2) for t in range(2)]
    return torch.cat(taps, dim=-1).reshape(N * (h + 1) * (w + 1), 4 * C)


def upsample_conv_phase(x: torch.Tensor, wg: torch.Tensor) -> torch.Tensor:
    """conv3x3(nearest_x2(x)) without bias, in the phase layout: [N, 4C, h+1, w+1] channels-last
    (memory [N, h+1, w+1, 4C]); ``wg`` from ``phase_gemm_weights``."""
    N, C, h, w = x.shape
    cout = wg.shape[0] // 4
    t = F.linear(im2col2x2(x), wg)  # [N*(h+1)*(w+1), 4*cout]
    return t.view(N, h + 1, w + 1, 4 * cout).permute(0, 3, 1, 2)


def phase_to_dense(t: torch.Tensor, hw: tuple, bias: torch.Tensor | None = None) -> torch.Tensor:
    """Phase layout [N, 4C, h+1, w+1] (+ bias [C]) -> dense [N, C, 2h, 2w] channels-last."""
    N, C4, hp, wp = t.shape
    C, (H, W) = C4 // 4, hw
    assert H == 2 * (hp - 1) and W == 2 * (wp - 1), (t.shape, hw)
    if (_lib.use_native(t, bias) and _nhwc(t) and C % 8 == 0 and t.data_ptr() % 16 == 0
            and _lib.has("kca_phase_to_dense_nhwc")):
        out = torch.empty(N, H, W, C, device=t.device, dtype=t.dtype)
        _lib.call("kca_phase_to_dense_nhwc", t.data_ptr(), _lib.ptr(bias.contiguous() if bias is not None else None),
                  out.data_ptr(), N, hp - 1, wp - 1, C, _lib.stream())
        return out.permute(0, 3, 1, 2)
    out = t.new_empty(N, C, H, W)
    for a in range(2):
        for b in range(2):
            k = 2 * a + b
            out[:, :, a::2, b::2] = t[:, k * C:(k + 1) * C, a:a + H // 2, b:b + W // 2]
    if bias is not None:
        out = out + bias.to(out.dtype)[None, :, None, None]
    return out.contiguous(memory_format=torch.channels_last)


def upsample_nearest2x(x: torch.Tensor) -> torch.Tensor:
    """Nearest x2 of a channels-last [N, C, h, w] tensor (native NHWC kernel on the GPU)."""
    N, C, h, w = x.shape
    if native_ok(x) and _lib.has("kca_upsample2x_nhwc"):
        out = torch.empty(N, 2 * h, 2 * w, C, device=x.device, dtype=x.dtype)
        _lib.call("kca_upsample2x_nhwc", x.data_ptr(), out.data_ptr(), N, h, w, C, _lib.stream())
        return out.permute(0, 3, 1, 2)
    return F.interpolate(x, scale_factor=2.0, mode="nearest")


class _UpsampleConvPhaseFn(torch.autograd.Function):
    """Training form of ``conv3x3(nearest_x2(x)) + bias`` as im2col + GEMM + dense scatter
    (channels-last bf16 on the GPU): backward = phase gather of the output gradient
    (``kca_dense_to_phase_nhwc``), the bias gradient as its column sum, dWg = dT^T A (A recomputed
    from x rather than saved), dA = dT Wg and dx = col2im(dA) (``kca_col2im2x2_nhwc``). The phase
    weights' gradient flows to the 3x3 kernel through ``phase_gemm_weights`` (torch ops)."""

    @staticmethod
    def forward(ctx, x, wg, bias):
        N, C, h, w = x.shape
        t = F.linear(im2col2x2(x), wg)
        ctx.save_for_backward(x, wg)
        ctx.has_bias = bias is not None
        out = phase_to_dense(t.view(N, h + 1, w + 1, -1).permute(0, 3, 1, 2), (2 * h, 2 * w), bias)
        return out

    @staticmethod
    def backward(ctx, dout):
        from .linear import column_sum
        x, wg = ctx.saved_tensors
        N, C, h, w = x.shape
        cout = wg.shape[0] // 4
        d = dout.contiguous(memory_format=torch.channels_last)
        dt = torch.empty(N * (h + 1) * (w + 1), 4 * cout, device=x.device, dtype=x.dtype)
        _lib.call("kca_dense_to_phase_nhwc", d.data_ptr(), dt.data_ptr(), N, h, w, cout, _lib.stream())
        db = column_sum(d.permute(0, 2, 3, 1).reshape(-1, cout)) if ctx.has_bias else None
        dwg = dx = None
        if ctx.needs_input_grad[1]:
            dwg = dt.t() @ im2col2x2(x)
        if ctx.needs_input_grad[0]:
            da = dt @ wg
            dxn = torch.empty(N, h, w, C, device=x.device, dtype=x.dtype)
            _lib.call("kca_col2im2x2_nhwc", da.data_ptr(), dxn.data_ptr(), N, h, w, C, _lib.stream())
            dx = dxn.permute(0, 3, 1, 2)
        return dx, dwg, db


def upsample_conv_train(x: torch.Tensor, w3: torch.Tensor, bias: torch.Tensor | None) -> torch.Tensor:
    """``conv3x3(nearest_x2(x), w3, bias, padding=1)`` with autograd through the phase GEMM on the
    GPU (channels-last bf16, C % 8 == 0); the plain form otherwise."""
    if (native_ok(x) and w3.shape[0] % 8 == 0 and _lib.has("kca_col2im2x2_nhwc")
            and (bias is None or bias.dtype == x.dtype)):
        return _UpsampleConvPhaseFn.apply(x, phase_gemm_weights(w3), bias)
    return F.conv2d(F.interpolate(x, scale_factor=2.0, mode="nearest"), w3, bias, padding=1)


__all__ = ["upsample_conv_train", "phase_weights", "phase_gemm_weights", "im2col2x2", "upsample_conv_phase",
           "phase_to_dense", "upsample_nearest2x"]
