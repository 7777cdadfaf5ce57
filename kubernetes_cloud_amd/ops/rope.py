"""Rotary position embedding (K3): GPT-J interleaved and NeoX rotate-half.

``apply_rotary_(q, k, ...)`` rotates the first ``rot`` dims of every head *in
place*, on strided [tokens, heads, head_dim] views (e.g. the fused QKV GEMM
output), so no copy of Q/K is made. It is used inside the attention autograd
function, which applies the transpose rotation to dQ/dK in its backward.
"""
from __future__ import annotations

import math

import torch

from . import _lib

_TABLES: dict = {}


def rope_tables(rot: int, max_pos: int, base: float = 10000.0, device=None):
    """fp32 cos/sin tables [max_pos, rot/2] (HF: inv_freq = base^(-2i/rot))."""
    key = (rot, max_pos, base, str(device))
    t = _TABLES.get(key)
    if t is None:
        inv = 1.0 / (base ** (torch.arange(0, rot, 2, dtype=torch.float64) / rot))
        pos = torch.arange(max_pos, dtype=torch.float64)
        ang = torch.outer(pos, inv)
        t = (ang.cos().float().to(device), ang.sin().float().to(device))
        _TABLES[key] = t
    return t


def _rotate_ref(x: torch.Tensor, cos: torch.Tensor, sin: torch.Tensor, interleaved: bool,
                sign: float):
    """x: [T, H, D] (any float dtype); rotates x[..., :rot] in fp32, returns new tensor."""
    rot = cos.shape[-1] * 2
    xf = x.float()
    xr = xf[..., :rot]
    c = cos[:, None, :]
    s = sin[:, None, :] * sign
    if interleaved:
        a, b = xr[..., 0::2], xr[..., 1::2]
        oa, ob = a * c - b * s, b * c + a * s
        out = torch.stack((oa, ob), dim=-1).flatten(-2)
    else:
        half = rot // 2
        a, b = xr[..., :half], xr[..., half:]
        out = torch.cat((a * c - b * s, b * c + a * s), dim=-1)
    res = torch.cat((out, xf[..., rot:]), dim=-1) if rot < x.shape[-1] else out
    return res.to(x.dtype)


def apply_rotary_(q: torch.Tensor, k: torch.Tensor, rot: int, seq: int, interleaved: bool,
                  base: float = 10000.0, sign: float = 1.0, pos_ids: torch.Tensor | None = None,
                  max_pos: int | None = None):
    """In-place rotation of q: [B, S, Hq, D] and k: [B, S, Hk, D] strided views.

    Token dims (B, S) must be collapsible to one stride (true for views into a
    [B*S, n*D] GEMM output).
    """
    if rot <= 0:
        return
    B, S = q.shape[0], q.shape[1]
    tokens = B * S
    mp = max_pos or max(seq, 1)
    if pos_ids is not None:
        mp = max(mp, int(pos_ids.max().item()) + 1)
    cos, sin = rope_tables(rot, mp, base, q.device)
    if _lib.use_native(q, k):
        assert q.stride(0) == S * q.stride(1) and k.stride(0) == S * k.stride(1)
        assert q.stride(-1) == 1 and k.stride(-1) == 1
        pid = pos_ids.to(torch.int32).contiguous() if pos_ids is not None else None
        _lib.call("kca_rope", q.data_ptr(), k.data_ptr(), q.shape[2], k.shape[2], tokens, S,
                  q.stride(1), q.stride(2), k.stride(1), k.stride(2), rot, int(interleaved),
                  cos.data_ptr(), sin.data_ptr(), _lib.ptr(pid), float(sign), _lib.stream())
        return
    if pos_ids is None:
        pos = torch.arange(S, device=q.device).repeat(B)
    else:
        pos = pos_ids.reshape(-1).to(q.device)
    c, s = cos[pos], sin[pos]
    for t in (q, k):
        flat = t.reshape(tokens, t.shape[2], t.shape[3]) if t.is_contiguous() else None
        src = t.reshape(tokens, t.shape[2], t.shape[3])
        out = _rotate_ref(src, c, s, interleaved, sign)
        if flat is not None:
            flat.copy_(out)
        else:
            t.copy_(out.view(t.shape))


def rotary_reference(x: torch.Tensor, rot: int, interleaved: bool, base: float = 10000.0):
    """Out-of-place reference for tests: x [B, S, H, D]."""
    B, S, H, D = x.shape
    cos, sin = rope_tables(rot, S, base, x.device)
    pos = torch.arange(S, device=x.device).repeat(B)
    out = _rotate_ref(x.reshape(B * S, H, D), cos[pos], sin[pos], interleaved, 1.0)
    return out.view(B, S, H, D)


__all__ = ["apply_rotary_", "rope_tables", "rotary_reference", "math"]
