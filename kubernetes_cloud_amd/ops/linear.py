"""Linear layers whose backward runs both GEMMs in the K-contiguous ("TN") layout.

PyTorch's Linear backward issues dX = dY W as an NN GEMM and dW = dY^T X as an
NT GEMM; on MI355X (hipBLASLt, GPT-J shapes, profiles/gemm_layout_gptj_r1.jsonl)
those run at 1.21-1.31 and 1.10-1.15 PFLOP/s, against 1.43-1.54 for the same
math with both operands K-contiguous. ``TLinear`` keeps a transposed copy of
its weight (refreshed after every optimizer step: ~4.5 ms for GPT-J-6B) for
dX = F.linear(dY, W^T), and transposes dY and X with ``kca_transpose_bf16``
(HBM-speed, csrc/kernels/transpose.hip) so that dW = F.linear(dY^T, X^T).
CPU tensors and inference use plain ``F.linear``.
"""
from __future__ import annotations

import torch
import torch.nn as nn
import torch.nn.functional as F

from . import _lib


def transpose(x: torch.Tensor) -> torch.Tensor:
    """[R, C] -> contiguous [C, R]; native for bf16 GPU tensors with R, C % 8 == 0."""
    R, C = x.shape
    if (_lib.use_native(x) and R % 8 == 0 and C % 8 == 0 and x.stride(1) == 1 and x.stride(0) % 8 == 0
            and x.data_ptr() % 16 == 0):
        out = torch.empty(C, R, device=x.device, dtype=x.dtype)
        _lib.call("kca_transpose_bf16", x.data_ptr(), x.stride(0), out.data_ptr(), R, R, C, _lib.stream())
        return out
    return x.t().contiguous()


def _tn_ok(t: torch.Tensor) -> bool:
    return t.shape[0] % 8 == 0 and t.shape[1] % 8 == 0


class _LinearTN(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, bias, layer):
        y = F.linear(x, weight, bias)
        ctx.save_for_backward(x, weight)
        ctx.layer = layer
        ctx.has_bias = bias is not None
        return y

    @staticmethod
    def backward(ctx, dy):
        x, weight = ctx.saved_tensors
        K, N = x.shape[-1], dy.shape[-1]
        x2 = x.reshape(-1, K)
        dy2 = dy.reshape(-1, N).contiguous()
        dx = dw = db = None
        if ctx.needs_input_grad[0]:
            wt = ctx.layer.weight_t
            dx = (F.linear(dy2, wt) if wt is not None else dy2 @ weight).view(x.shape)
        if ctx.needs_input_grad[1]:
            if _tn_ok(dy2) and _tn_ok(x2):
                dw = F.linear(transpose(dy2), transpose(x2))
            else:
                dw = dy2.t() @ x2
        if ctx.has_bias and ctx.needs_input_grad[2]:
            db = dy2.sum(0)
        return dx, dw, db, None


class _ParamLinear(torch.autograd.Function):
    """y = x W^T + b that saves the Parameter W itself for backward. F.linear
    saves ``W.t()`` -- a view that pins W's storage at forward time; ZeRO-3
    (train/engine.py) swaps a released parameter's storage out after forward
    and back in (re-gathered) before backward, which only works when the
    autograd graph refers to the Parameter."""

    @staticmethod
    def forward(ctx, x, weight, bias):
        ctx.save_for_backward(x, weight)
        ctx.has_bias = bias is not None
        return F.linear(x, weight, bias)

    @staticmethod
    def backward(ctx, dy):
        x, weight = ctx.saved_tensors
        K, N = x.shape[-1], dy.shape[-1]
        x2 = x.reshape(-1, K)
        dy2 = dy.reshape(-1, N)
        dx = dw = db = None
        if ctx.needs_input_grad[0]:
            dx = (dy2 @ weight).view(x.shape)
        if ctx.needs_input_grad[1]:
            dw = dy2.t() @ x2
        if ctx.has_bias and ctx.needs_input_grad[2]:
            db = dy2.sum(0)
        return dx, dw, db


def param_linear(x, weight, bias=None):
    if torch.is_grad_enabled() and (x.requires_grad or weight.requires_grad):
        return _ParamLinear.apply(x, weight, bias)
    return F.linear(x, weight, bias)


class TLinear(nn.Linear):
    """nn.Linear (same parameters / state dict) with the TN backward above when
    ``enable_tn(True)`` was called and the input is a bf16 GPU tensor."""

    weight_t: torch.Tensor | None

    def __init__(self, *a, **kw):
        super().__init__(*a, **kw)
        self.weight_t = None
        self._tn = False

    def enable_tn(self, on: bool = True):
        # any 8-aligned shape: dX runs TN off weight_t, dW TN on transposed dY / X (edge tiles of
        # the transpose kernel cover GPT-J's 50400-row LM head: 12.2 ms NT per micro-batch before)
        self._tn = bool(on) and self.weight.is_cuda and self.weight.dtype == torch.bfloat16 \
            and self.weight.shape[0] % 8 == 0 and self.weight.shape[1] % 8 == 0
        self.weight_t = torch.empty(self.weight.shape[1], self.weight.shape[0], device=self.weight.device,
                                    dtype=self.weight.dtype) if self._tn else None
        self.refresh_transposed()

    @torch.no_grad()
    def refresh_transposed(self):
        if self.weight_t is not None:
            w = self.weight.detach()
            if not _tn_ok(w):
                self.weight_t.copy_(w.t())
                return
            _lib.call("kca_transpose_bf16", w.data_ptr(), w.stride(0), self.weight_t.data_ptr(), w.shape[0],
                      w.shape[0], w.shape[1], _lib.stream())

    def forward(self, x):
        if self._tn and torch.is_grad_enabled() and (x.requires_grad or self.weight.requires_grad) \
                and x.is_cuda and x.dtype == torch.bfloat16:
            return _LinearTN.apply(x, self.weight, self.bias, self)
        return F.linear(x, self.weight, self.bias)


__all__ = ["TLinear", "transpose", "param_linear"]


# ---------------------------------------------------------------- split-K weight gradients
def _wgrad_splits(tokens: int, n: int, k: int) -> int:
    """Token chunks for dW = dY^T X: one hipBLASLt GEMM leaves most CUs idle when the output is
    small and the token (reduction) dimension long (SD UNet linears: 320x320 over 65536 tokens ran
    at ~90 TFLOP/s). Split into a batched GEMM over token chunks + an fp32 sum: 320x320 / 65536
    0.131 -> 0.065 ms, 640x640 / 16384 0.076 -> 0.052 ms, 320x1280 / 65536 0.179 -> 0.103 ms
    (bench/wgrad_splitk_bench.py, profiles/wgrad_splitk_r2.jsonl); 5120x640 is faster unsplit."""
    if tokens < 16384 or n * k > 1_700_000:
        return 1
    s = min(16, tokens // 2048)
    while s > 1 and tokens % s:
        s //= 2
    return s


_COLSUM = __import__("os").environ.get("KCA_COLSUM", "1") not in ("0", "false")  # A/B knob


def column_sum(x2: torch.Tensor, out_dtype: torch.dtype | None = None) -> torch.Tensor:
    """Sum over the rows of a [M, N] tensor (a bias gradient), in ``out_dtype`` (default x2's):
    ``kca_colsum_bf16`` (row-chunk partials, then a small fp32 sum) for contiguous bf16 on the GPU."""
    M, N = x2.shape
    out_dtype = out_dtype or x2.dtype
    if not (_COLSUM and _lib.use_native(x2) and x2.dtype == torch.bfloat16 and x2.is_contiguous() and N % 8 == 0
            and x2.data_ptr() % 16 == 0 and _lib.has("kca_colsum_bf16")):
        return x2.sum(0) if out_dtype == x2.dtype else x2.sum(0, dtype=torch.float32).to(out_dtype)
    rb = max(64, -(-M // 256) // 8 * 8)  # ~256 row chunks
    nb = -(-M // rb)
    part = torch.empty(nb, N, device=x2.device, dtype=torch.float32)
    _lib.call("kca_colsum_bf16", x2.data_ptr(), part.data_ptr(), M, N, rb, _lib.stream())
    return sum_parts(part, out_dtype)


def sum_parts(part: torch.Tensor, out_dtype: torch.dtype) -> torch.Tensor:
    """[S, *shape] fp32 partials -> their sum over S in ``out_dtype`` (bf16 / fp32): one native pass
    (``kca_col_reduce_f32``) instead of torch's sum + cast."""
    S = part.shape[0]
    C = part[0].numel()
    if (part.is_cuda and part.dtype == torch.float32 and part.is_contiguous() and C % 64 == 0
            and out_dtype in (torch.bfloat16, torch.float32) and _lib.has("kca_col_reduce_f32")):
        out = torch.empty(part.shape[1:], device=part.device, dtype=out_dtype)
        bf = out_dtype == torch.bfloat16
        _lib.call("kca_col_reduce_f32", part.data_ptr(), S, C, out.data_ptr() if bf else None,
                  None if bf else out.data_ptr(), _lib.stream())
        return out
    return part.sum(0).to(out_dtype)


_BMM_F32 = [None]  # aten::bmm.dtype (bf16 in, fp32 out): probed on first use


def _bmm_f32(a: torch.Tensor, b: torch.Tensor) -> torch.Tensor:
    if _BMM_F32[0] is not False and a.is_cuda and a.dtype == torch.bfloat16:
        try:
            r = torch.bmm(a, b, out_dtype=torch.float32)
            _BMM_F32[0] = True
            return r
        except (TypeError, RuntimeError, NotImplementedError):
            _BMM_F32[0] = False
    return torch.bmm(a, b).float()


class _LinearSplitKW(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, bias):
        ctx.save_for_backward(x, weight)
        ctx.has_bias = bias is not None
        return F.linear(x, weight, bias)

    @staticmethod
    def backward(ctx, gy):
        x, w = ctx.saved_tensors
        n, k = w.shape
        gy2 = gy.reshape(-1, n)
        x2 = x.reshape(-1, k)
        gx = gw = gb = None
        if ctx.needs_input_grad[0]:
            gx = (gy2 @ w).view(x.shape)
        if ctx.needs_input_grad[1]:
            t = gy2.shape[0]
            s = _wgrad_splits(t, n, k)
            if s > 1:
                gy2c = gy2 if gy2.is_contiguous() else gy2.contiguous()
                x2c = x2 if x2.is_contiguous() else x2.contiguous()
                # per-chunk products in fp32 straight from the GEMM, one native reduction to w's dtype
                gw = sum_parts(_bmm_f32(gy2c.view(s, t // s, n).transpose(1, 2), x2c.view(s, t // s, k)), w.dtype)
            else:
                gw = gy2.t() @ x2
        if ctx.has_bias and ctx.needs_input_grad[2]:
            gb = column_sum(gy2 if gy2.is_contiguous() else gy2.contiguous())
        return gx, gw, gb


def linear_splitk_wgrad(x: torch.Tensor, weight: torch.Tensor, bias: torch.Tensor | None = None) -> torch.Tensor:
    """F.linear whose weight gradient splits long token reductions (see _wgrad_splits); plain
    F.linear when no gradient is recorded or off the GPU."""
    if not (torch.is_grad_enabled() and x.is_cuda and weight.requires_grad):
        return F.linear(x, weight, bias)
    return _LinearSplitKW.apply(x, weight, bias)


class SplitKLinear(nn.Linear):
    """nn.Linear (same parameters / state-dict keys) training through linear_splitk_wgrad."""

    def forward(self, x):
        return linear_splitk_wgrad(x, self.weight, self.bias)


_WS: dict[int, torch.Tensor] = {}
_WS_BYTES = 32 << 20


def _workspace(dev: torch.device) -> torch.Tensor | None:
    """hipBLASLt workspace, allocated once per device outside any graph capture."""
    ws = _WS.get(dev.index)
    if ws is None and not torch.cuda.is_current_stream_capturing():
        ws = _WS[dev.index] = torch.empty(_WS_BYTES, device=dev, dtype=torch.uint8)
    return ws


class _LinearResidualFn(torch.autograd.Function):
    """Training ``res + F.linear(x, W, b)``: the forward is the one-GEMM epilogue form; the backward
    passes dY through to ``res`` (no copy), dX = dY W, dW by the split-K weight gradient, db by the
    column-sum kernel -- the residual add's separate read-read-write pass is gone."""

    @staticmethod
    def forward(ctx, x, weight, bias, res):
        with torch.no_grad():
            y = linear_residual(x, weight, bias, res)
        ctx.save_for_backward(x, weight)
        ctx.has_bias = bias is not None
        return y

    @staticmethod
    def backward(ctx, gy):
        x, w = ctx.saved_tensors
        gb = None
        gx, gw, gb0 = _LinearSplitKW.backward(_Saved(x, w, ctx.has_bias, ctx.needs_input_grad[:3]), gy)
        if ctx.has_bias and ctx.needs_input_grad[2]:
            gb = gb0
        return gx, gw, gb, (gy if ctx.needs_input_grad[3] else None)


class _Saved:
    """ctx stand-in for reusing _LinearSplitKW.backward."""

    def __init__(self, x, w, has_bias, needs):
        self.saved_tensors = (x, w)
        self.has_bias = has_bias
        self.needs_input_grad = tuple(needs)


def linear_residual_train(x: torch.Tensor, weight: torch.Tensor, bias: torch.Tensor | None,
                          res: torch.Tensor) -> torch.Tensor:
    """``res + F.linear(x, weight, bias)`` with autograd, fused on the GPU (see _LinearResidualFn)."""
    if torch.is_grad_enabled() and _lib.use_native(x, weight, res) and res.stride(-1) == 1 and x.stride(-1) == 1:
        return _LinearResidualFn.apply(x, weight, bias, res)
    return linear_residual(x, weight, bias, res)


def linear_residual(x: torch.Tensor, weight: torch.Tensor, bias: torch.Tensor | None,
                    res: torch.Tensor) -> torch.Tensor:
    """``res + F.linear(x, weight, bias)`` in ONE hipBLASLt GEMM (bias and residual in its epilogue,
    csrc/kernels/gemm_lt.hip) at inference on the GPU; the two-pass form otherwise (autograd,
    CPU). ``res`` is any view whose rows are the output rows ([..., N], unit last stride); the
    result has ``res``'s shape."""
    N, K = weight.shape
    if not (not torch.is_grad_enabled() and _lib.use_native(x, weight, res) and (bias is None or bias.is_cuda)
            and x.shape[-1] == K and res.shape[-1] == N and x.stride(-1) == 1 and res.stride(-1) == 1
            and weight.stride(1) == 1 and (bias is None or bias.is_contiguous())):
        return res + F.linear(x, weight, bias).reshape(res.shape)
    x2 = x.reshape(-1, K)
    r2 = res.reshape(-1, N)
    M = x2.shape[0]
    if r2.shape[0] != M or x2.stride(1) != 1 or r2.stride(1) != 1:
        return res + F.linear(x, weight, bias).reshape(res.shape)
    out = torch.empty(M, N, device=x.device, dtype=x.dtype)
    ws = _workspace(x.device)
    _lib.call("kca_gemm_lt", x2.data_ptr(), x2.stride(0), weight.data_ptr(), weight.stride(0), _lib.ptr(bias),
              r2.data_ptr(), r2.stride(0), out.data_ptr(), N, M, N, K, 1.0, _lib.ptr(ws),
              _WS_BYTES if ws is not None else 0, _lib.stream())
    return out.view(res.shape)
