"""Skinny (decode) GEMM: y = act(x W^T + b) for x with <= 16 rows.

``kca_skinny_gemm`` (csrc/kernels/gemv.hip) streams W once at HBM speed with
bias + GELU fused in the store; used by the serving runner for every decode
linear (QKV, out-proj, fc_in+GELU, fc_out, LM head). Larger M goes to
hipBLASLt through ``F.linear``.
"""
from __future__ import annotations

import os

import torch
import torch.nn.functional as F

from . import _lib

ACT = {None: 0, "none": 0, "tanh": 1, "gelu_tanh": 1, "erf": 2, "none_erf": 2}


def _act_ref(y, act):
    if act == 1:
        return F.gelu(y.float(), approximate="tanh").to(y.dtype)
    if act == 2:
        return F.gelu(y.float()).to(y.dtype)
    return y


_MODE_SET = False


def _set_mode():
    """KCA_SKINNY_SPLITK=0 selects the row-per-wave kernel (A/B runs)."""
    global _MODE_SET
    if not _MODE_SET:
        _MODE_SET = True
        if os.environ.get("KCA_SKINNY_SPLITK", "1") in ("0", "false") and _lib.has("kca_skinny_set_splitk"):
            _lib.call("kca_skinny_set_splitk", 0)
        r = int(os.environ.get("KCA_GEMV_SMALLK_R", "0"))
        if r and _lib.has("kca_skinny_set_smallk"):
            _lib.call("kca_skinny_set_smallk", r)


# rows up to which every weight streams through the skinny kernel (A/B knob): M = 1 and M = 2 run the
# register-resident K-split GEMV (B=2 GPT-J decode 3.13-3.16 vs 3.41-3.50 ms/step through hipBLASLt);
# from 3 rows hipBLASLt is faster on the big weights (profiles/decode_skinny_ab_r2.txt)
_SKINNY_MAX_M = int(os.environ.get("KCA_SKINNY_MAX_M", "2"))


def skinny_linear(x: torch.Tensor, weight: torch.Tensor, bias: torch.Tensor | None = None, act: int = 0,
                  out: torch.Tensor | None = None) -> torch.Tensor:
    """x [M, K] (row stride multiple of 8), weight [N, K] contiguous."""
    M, K = x.shape
    N = weight.shape[0]
    # measured on MI355X (profiles/gemv_bench_r1.jsonl, decode_bench in context): the skinny kernel wins
    # at M = 1 and for 2 <= M <= 4 only on the small out-projection (hipBLASLt under-fills the chip there:
    # 12.4 vs 18.4 us); on the QKV / MLP weights hipBLASLt is faster from M = 2 (GPT-J decode B=2 4.69 ms
    # with the skinny kernel vs 4.54 ms at B=4 through hipBLASLt); MFMA GEMMs beyond
    small = N * K <= (16 << 20)
    # M = 2 takes the register-resident K-split form only for K <= 8192 (GPT-J); BLOOM's K = 14336
    # QKV / fc_in at M = 2 would fall to the row-per-wave kernel, which hipBLASLt beats on big weights
    regs = M == 1 or K <= 8192 or small
    if M == 1 and _lib.native_f16(x, weight) and K % 8 == 0 and weight.is_contiguous() \
            and x.data_ptr() % 16 == 0 and weight.data_ptr() % 16 == 0 and (bias is None or bias.dtype == x.dtype):
        # fp16 (FT / DS-Inference serving precision): the single-row GEMV's fp16 instantiation
        if out is None:
            out = torch.empty(M, N, device=x.device, dtype=x.dtype)
        _lib.call("kca_skinny_gemm_f16", x.data_ptr(), x.stride(0), weight.data_ptr(), _lib.ptr(bias),
                  out.data_ptr(), out.stride(0), M, N, K, int(act), _lib.stream())
        return out
    if (_lib.use_native(x, weight) and ((M <= _SKINNY_MAX_M and regs) or (M <= 4 and small)) and K % 8 == 0
            and x.stride(1) == 1
            and x.stride(0) % 8 == 0
            and weight.is_contiguous() and x.data_ptr() % 16 == 0 and weight.data_ptr() % 16 == 0
            and (bias is None or bias.dtype == torch.bfloat16)):
        _set_mode()
        if out is None:
            out = torch.empty(M, N, device=x.device, dtype=x.dtype)
        _lib.call("kca_skinny_gemm", x.data_ptr(), x.stride(0), weight.data_ptr(), _lib.ptr(bias), out.data_ptr(),
                  out.stride(0), M, N, K, int(act), _lib.stream())
        return out
    y = _linear_act(x, weight, bias, act)
    if out is not None:
        out.copy_(y)
        return out
    return y


# hipBLASLt decode linears with an activation (M > the skinny kernel's rows: fc_in at B >= 3): the
# GELU as ONE native in-place pass (kca_gelu_fwd) instead of three eager kernels (to fp32, gelu,
# to bf16: ~25 us per layer at B = 32, on the MLP branch's critical path)
def _linear_act(x, weight, bias, act):
    if not act:
        return F.linear(x, weight, bias)
    y = F.linear(x, weight, bias)
    f16 = _lib.native_f16(y) and _lib.has("kca_gelu_fwd_f16")
    if (_lib.use_native(y) or f16) and y.is_contiguous() and y.numel() % 8 == 0 and y.data_ptr() % 16 == 0 \
            and y.dtype in (torch.bfloat16, torch.float16):
        _lib.call("kca_gelu_fwd_f16" if f16 else "kca_gelu_fwd", y.data_ptr(), y.data_ptr(), y.numel(),
                  int(act == 1), _lib.stream())
        return y
    return _act_ref(y, act)


def _ln_ok(x, M, K, weight, residuals, gamma, beta, bias):
    Mp = 1 if M == 1 else 2 if M == 2 else 4 if M <= 4 else 8
    ts = [x, weight, gamma, *residuals] + ([beta] if beta is not None else [])
    return (M == 1 or (M <= 4 and weight.shape[0] * K <= (16 << 20))) and Mp * K <= 32768 and K % 8 == 0 \
        and all(t.data_ptr() % 16 == 0 for t in ts) and x.stride(1) == 1 and x.stride(0) % 8 == 0 \
        and all(r.is_contiguous() and r.shape == x.shape for r in residuals) and weight.is_contiguous() \
        and gamma.is_contiguous() and (beta is None or beta.is_contiguous()) \
        and (bias is None or bias.dtype == torch.bfloat16)


# M == 1: normalise once (ln_fwd_kernel, one workgroup) and stream the weights with the plain GEMV,
# instead of every GEMV workgroup re-reading x + residuals + gamma/beta and redoing the reductions
# (at N = 12288 that per-workgroup prologue moved more L2 bytes than the weights themselves).
_LN_SPLIT_M1 = os.environ.get("KCA_DECODE_LN_SPLIT", "1") not in ("0", "false")


def ln_rows(x: torch.Tensor, gamma: torch.Tensor, beta: torch.Tensor | None, eps: float, residuals=()):
    """Decode LayerNorm alone: ``(xn, h)`` with h = x + sum(residuals) (bf16-rounded)
    and xn = LN(h) -- ``kca_ln_rows`` (one register-resident workgroup per row)."""
    M, K = x.shape
    residuals = tuple(r for r in residuals if r is not None)
    f16 = _lib.native_f16(x, gamma)
    if (_lib.use_native(x) or f16) and K % 8 == 0 and K <= 16384 and x.stride(1) == 1 and x.stride(0) % 8 == 0 \
            and all(r.is_contiguous() and r.shape == x.shape for r in residuals) and len(residuals) <= 2 \
            and gamma.is_contiguous() and (beta is None or beta.is_contiguous()):
        h = torch.empty(M, K, device=x.device, dtype=x.dtype) if residuals else x
        xn = torch.empty(M, K, device=x.device, dtype=x.dtype)
        r1 = residuals[0] if residuals else None
        r2 = residuals[1] if len(residuals) > 1 else None
        _lib.call("kca_ln_rows_f16" if f16 else "kca_ln_rows", x.data_ptr(), x.stride(0), _lib.ptr(r1), _lib.ptr(r2),
                  h.data_ptr() if residuals else None, h.stride(0) if residuals else K, gamma.data_ptr(),
                  _lib.ptr(beta), float(eps), xn.data_ptr(), M, K, _lib.stream())
        return xn, h
    from .norms import layer_norm
    if residuals:
        return layer_norm(x, gamma, beta, eps, residual=residuals)
    return layer_norm(x, gamma, beta, eps), x


def embed_ln_rows(wte: torch.Tensor, tokens: torch.Tensor, gamma: torch.Tensor, beta: torch.Tensor | None,
                  eps: float, chain: torch.Tensor | None = None, prev: torch.Tensor | None = None):
    """Decode step head: ``(xn, h)`` with h[m] = wte[id_m] and xn = LN(h), id_m = prev[chain[m]] where
    chain[m] >= 0 (a token sampled by the previous step, still on the device) else tokens[m] --
    one launch (``kca_embed_ln_rows``) instead of the embedding gather, the position cast and the LN."""
    M, K = tokens.shape[0], wte.shape[1]
    f16 = _lib.native_f16(wte, gamma)
    if not ((_lib.use_native(wte) or f16) and K % 8 == 0 and K <= 16384 and wte.stride(1) == 1 and wte.stride(0) % 8 == 0
            and gamma.is_contiguous() and (beta is None or beta.is_contiguous()) and tokens.dtype == torch.int64):
        ids = tokens
        if chain is not None:
            ids = torch.where(chain >= 0, prev[chain.clamp(min=0).long()], tokens)
        return ln_rows(wte[ids], gamma, beta, eps)
    h = torch.empty(M, K, device=wte.device, dtype=wte.dtype)
    xn = torch.empty(M, K, device=wte.device, dtype=wte.dtype)
    _lib.call("kca_embed_ln_rows_f16" if f16 else "kca_embed_ln_rows", wte.data_ptr(), wte.stride(0), tokens.data_ptr(), _lib.ptr(chain), _lib.ptr(prev),
              wte.shape[0], h.data_ptr(), K, gamma.data_ptr(), _lib.ptr(beta), float(eps), xn.data_ptr(), M, K,
              _lib.stream())
    return xn, h


def ln_skinny_linear(x: torch.Tensor, gamma: torch.Tensor, beta: torch.Tensor | None, eps: float,
                     weight: torch.Tensor, bias: torch.Tensor | None = None, residuals=(), act: int = 0,
                     want_h: bool = False, want_xn: bool = False):
    """``act(LayerNorm(x + sum(residuals)) W^T + b)`` in one launch (decode).

    Returns ``(y, h)`` with ``h`` the updated residual stream (``x`` itself when
    no residuals are added), plus the normalised rows ``xn`` when ``want_xn``
    (GPT-J's shared LayerNorm feeds a second GEMM). Falls back to the LN
    kernel + ``skinny_linear`` when the rows do not fit the LDS tile or the
    batch is too wide."""
    M, K = x.shape
    residuals = tuple(r for r in residuals if r is not None)
    split = M == 1 and _LN_SPLIT_M1  # one LN launch + the plain GEMV (A/B knob, see _LN_SPLIT_M1)
    if not split and _lib.use_native(x, weight) and _ln_ok(x, M, K, weight, residuals, gamma, beta, bias):
        h = torch.empty(M, K, device=x.device, dtype=x.dtype) if residuals else x
        y = torch.empty(M, weight.shape[0], device=x.device, dtype=x.dtype)
        xn = torch.empty(M, K, device=x.device, dtype=x.dtype) if want_xn else None
        r1 = residuals[0] if residuals else None
        r2 = residuals[1] if len(residuals) > 1 else None
        _set_mode()
        _lib.call("kca_ln_skinny_gemm", x.data_ptr(), x.stride(0), _lib.ptr(r1), _lib.ptr(r2),
                  h.data_ptr() if residuals else None, h.stride(0) if residuals else K, gamma.data_ptr(),
                  _lib.ptr(beta), float(eps), weight.data_ptr(), _lib.ptr(bias), y.data_ptr(), y.stride(0),
                  M, weight.shape[0], K, int(act), _lib.ptr(xn), _lib.stream())
        return (y, h, xn) if want_xn else (y, h)
    if split:
        xn, h = ln_rows(x, gamma, beta, eps, residuals)
        y = skinny_linear(xn, weight, bias, act)
        return (y, h, xn) if want_xn else (y, h)
    if _lib.native_f16(x, gamma):  # fp16 rows: the register-resident LN kernel's fp16 instantiation
        xn, h = ln_rows(x, gamma, beta, eps, residuals)
    else:
        from .norms import layer_norm
        if residuals:
            xn, h = layer_norm(x, gamma, beta, eps, residual=residuals)
        else:
            xn, h = layer_norm(x, gamma, beta, eps), x
    y = skinny_linear(xn, weight, bias, act)
    return (y, h, xn) if want_xn else (y, h)


__all__ = ["skinny_linear", "ln_skinny_linear", "ln_rows", "ACT"]
