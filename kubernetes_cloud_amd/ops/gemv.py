"""Skinny (decode) GEMM: y = act(x W^T + b) for x with <= 16 rows.

``kca_skinny_gemm`` (csrc/kernels/gemv.hip) streams W once at HBM speed with
bias + GELU fused in the store; used by the serving runner for every decode
linear (QKV, out-proj, fc_in+GELU, fc_out, LM head). Larger M goes to
hipBLASLt through ``F.linear``.
"""
from __future__ import annotations

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


def skinny_linear(x: torch.Tensor, weight: torch.Tensor, bias: torch.Tensor | None = None, act: int = 0,
                  out: torch.Tensor | None = None) -> torch.Tensor:
    """x [M, K] (row stride multiple of 8), weight [N, K] contiguous."""
    M, K = x.shape
    N = weight.shape[0]
    # measured on MI355X (profiles/gemv_bench_r1.jsonl): the skinny kernel wins for M <= 2 everywhere and
    # up to M = 4 on small weights (hipBLASLt under-fills the chip there); MFMA GEMMs win beyond
    small = N * K <= (64 << 20)
    if (_lib.use_native(x, weight) and (M <= 2 or (M <= 4 and small)) and K % 8 == 0 and x.stride(1) == 1
            and x.stride(0) % 8 == 0
            and weight.is_contiguous() and x.data_ptr() % 16 == 0 and weight.data_ptr() % 16 == 0
            and (bias is None or bias.dtype == torch.bfloat16)):
        if out is None:
            out = torch.empty(M, N, device=x.device, dtype=x.dtype)
        _lib.call("kca_skinny_gemm", x.data_ptr(), x.stride(0), weight.data_ptr(), _lib.ptr(bias), out.data_ptr(),
                  out.stride(0), M, N, K, int(act), _lib.stream())
        return out
    y = _act_ref(F.linear(x, weight, bias), act)
    if out is not None:
        out.copy_(y)
        return out
    return y


__all__ = ["skinny_linear", "ACT"]
