"""Flash attention (K2/K13/K16) autograd ops over strided [B, S, H, D] views.

``flash_attention`` is the generic entry point (causal or not, GQA, ALiBi,
per-batch key lengths). ``qkv_rope_attention`` consumes the fused QKV GEMM
output in place: RoPE is applied to the Q/K slices by ``kca_rope`` and the
attention kernels read Q/K/V straight out of the [B, S, 3, H, D] buffer; the
backward writes dQ/dK/dV into one fused dQKV buffer (so one dgrad GEMM and one
wgrad GEMM serve all three projections) and un-rotates dQ/dK in place.

Masks: ``kv_len`` is None, int [B] key lengths (right padding), or a bool
[B, Sk] per-key mask with holes (the last context of a pad == eos dataset,
data/tokenized.py; finetuner.py:674-691) which the kernels take as a packed
bitmap; ``window`` > 0 is GPT-Neo's local band (key > q - window). CPU
tensors use the fp32 reference (``attention_reference``).
"""
from __future__ import annotations

import math

import torch

from . import _lib
from .rope import apply_rotary_


def attention_reference(q, k, v, causal: bool, scale: float | None = None,
                        kv_len: torch.Tensor | None = None, alibi: torch.Tensor | None = None,
                        window: int = 0):
    """fp32 reference. q [B,Sq,H,D], k/v [B,Sk,Hkv,D] -> o [B,Sq,H,D] (q.dtype), lse [B,H,Sq].
    ``kv_len``: int [B] key lengths (right padding), or a bool [B, Sk] per-key
    mask (True = attend) for masks with holes. ``window``: keys more than
    window-1 positions left of the (bottom-right aligned) query are masked."""
    B, Sq, H, D = q.shape
    Sk, Hkv = k.shape[1], k.shape[2]
    scale = scale if scale is not None else 1.0 / math.sqrt(D)
    qf = q.float().transpose(1, 2)
    kf = k.float().transpose(1, 2)
    vf = v.float().transpose(1, 2)
    if Hkv != H:
        rep = H // Hkv
        kf = kf.repeat_interleave(rep, dim=1)
        vf = vf.repeat_interleave(rep, dim=1)
    s = torch.matmul(qf, kf.transpose(-1, -2)) * scale
    qi = torch.arange(Sq, device=q.device)[:, None]
    ki = torch.arange(Sk, device=q.device)[None, :]
    off = Sk - Sq
    if alibi is not None:
        s = s + alibi.float().view(1, H, 1, 1) * (ki - qi - off).float()
    mask = torch.zeros(B, 1, Sq, Sk, dtype=torch.bool, device=q.device)
    if causal:
        mask = mask | (ki > qi + off)
    if window:
        mask = mask | (ki <= qi + off - window)
    if kv_len is not None and kv_len.dtype == torch.bool:  # per-key mask [B, Sk] (True = attend)
        mask = mask | ~kv_len.to(q.device).view(B, 1, 1, Sk)
    elif kv_len is not None:
        mask = mask | (ki[None, None] >= kv_len.view(B, 1, 1, 1).to(q.device))
    s = s.masked_fill(mask, float("-inf"))
    lse = torch.logsumexp(s, dim=-1)
    p = torch.exp(s - lse[..., None])
    p = torch.nan_to_num(p, nan=0.0)
    o = torch.matmul(p, vf).transpose(1, 2)
    return o.to(q.dtype), lse


def set_tiled_path(enable: bool) -> None:
    """Toggle the full-tile fast kernels (csrc/kernels/attention_tiled.hip) used
    for head_dim 128/256 when Sq % 128 == 0 and Sk % 32 (fwd) / 128 (bwd) == 0
    and there is no ALiBi / key-length mask. On by default; off forces the
    generic kernels (A/B measurement, tests)."""
    _lib.call("kca_attn_set_tiled", int(bool(enable)))


_VARIANT = [1]


def set_variant(v: int) -> int:
    """Full-tile kernel variants (A/B knob, attention_tiled.hip): bit 0 = the 8-wave D = 256
    forward (default on). Returns the previous value."""
    _lib.call("kca_attn_set_variant", int(v))
    old, _VARIANT[0] = _VARIANT[0], int(v)
    return old


def _strides(t):
    return t.stride(0), t.stride(1), t.stride(2)


def pack_key_mask(mask: torch.Tensor) -> torch.Tensor:
    """bool [B, Sk] (True = attend) -> int32 [B, ceil(Sk/32)] bitmap, bit k%32
    of word k//32 = key k (the kernels' ``key_mask``)."""
    B, Sk = mask.shape
    W = (Sk + 31) // 32
    m = torch.zeros(B, W * 32, dtype=torch.int64, device=mask.device)
    m[:, :Sk] = mask.to(torch.int64)
    words = (m.view(B, W, 32) << torch.arange(32, device=mask.device, dtype=torch.int64)).sum(-1)
    words = torch.where(words >= 2 ** 31, words - 2 ** 32, words)
    return words.to(torch.int32).contiguous()


def _masks(kv_len):
    """Internal mask form -> (lengths int32 [B] or None, bitmap int32 [B, W] or None)."""
    if kv_len is None:
        return None, None
    return (kv_len, None) if kv_len.dim() == 1 else (None, kv_len)


def _fwd(q, k, v, causal, scale, kv_len, alibi, out=None, window: int = 0, rowsum_col: int = -1,
         max_col: int = -1):
    B, Sq, H, D = q.shape
    Sk, Hkv = k.shape[1], k.shape[2]
    o = out if out is not None else torch.empty(B, Sq, H, D, device=q.device, dtype=q.dtype)
    lse = torch.empty(B, H, Sq, device=q.device, dtype=torch.float32)
    # overflow flags of the full-tile fast path (4 per 128-row block)
    flags = torch.empty(4 * ((Sq + 127) // 128) * B * H, device=q.device, dtype=torch.int32)
    lens, km = _masks(kv_len)
    _lib.call("kca_attn_fwd", q.data_ptr(), k.data_ptr(), v.data_ptr(), o.data_ptr(), lse.data_ptr(),
              *_strides(q), *_strides(k), *_strides(v), *_strides(o),
              B, Sq, Sk, H, Hkv, D, int(causal), float(scale), _lib.ptr(alibi), _lib.ptr(lens),
              int(window), _lib.ptr(km), int(rowsum_col), int(max_col), flags.data_ptr(), _lib.stream())
    return o, lse


def _bwd(q, k, v, o, do, lse, dq, dk, dv, causal, scale, kv_len, alibi, window: int = 0):
    B, Sq, H, D = q.shape
    Sk, Hkv = k.shape[1], k.shape[2]
    delta = torch.empty(B, H, Sq, device=q.device, dtype=torch.float32)
    _lib.call("kca_attn_bwd_preprocess", o.data_ptr(), do.data_ptr(), delta.data_ptr(),
              *_strides(o), *_strides(do), B, Sq, H, D, _lib.stream())
    _lib.call("kca_attn_bwd", q.data_ptr(), k.data_ptr(), v.data_ptr(), o.data_ptr(), do.data_ptr(),
              dq.data_ptr(), dk.data_ptr(), dv.data_ptr(), lse.data_ptr(), delta.data_ptr(),
              *_strides(q), *_strides(k), *_strides(v), *_strides(do),
              *_strides(dq), *_strides(dk), *_strides(dv),
              B, Sq, Sk, H, Hkv, D, int(causal), float(scale), _lib.ptr(alibi), _lib.ptr(_masks(kv_len)[0]),
              int(window), _lib.ptr(_masks(kv_len)[1]), _lib.stream())


def _check(q, k, v):
    for t in (q, k, v):
        if t.dim() != 4 or t.stride(-1) != 1:
            raise ValueError("attention expects [B, S, H, D] views with unit last stride")
        if t.dtype != torch.bfloat16:
            raise ValueError("native attention is bf16")
    D = q.shape[-1]
    if D % 8 or D > 256:
        raise ValueError(f"head_dim {D} unsupported (multiple of 8, <= 256)")


class _FlashAttnFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, q, k, v, causal, scale, kv_len, alibi, window):
        _check(q, k, v)
        o, lse = _fwd(q, k, v, causal, scale, kv_len, alibi, window=window)
        ctx.save_for_backward(q, k, v, o, lse, kv_len, alibi)
        ctx.causal, ctx.scale, ctx.window = causal, scale, window
        return o

    @staticmethod
    def backward(ctx, do):
        q, k, v, o, lse, kv_len, alibi = ctx.saved_tensors
        do = do.contiguous()
        dq = torch.empty(q.shape, device=q.device, dtype=q.dtype)
        dk = torch.empty(k.shape, device=k.device, dtype=k.dtype)
        dv = torch.empty(v.shape, device=v.device, dtype=v.dtype)
        _bwd(q, k, v, o, do, lse, dq, dk, dv, ctx.causal, ctx.scale, kv_len, alibi, ctx.window)
        return dq, dk, dv, None, None, None, None, None


def native_mask(kv_len, device):
    """Public mask form -> the kernels': int32 lengths [B], or the packed
    bitmap [B, W] of a bool per-key mask."""
    if kv_len is None:
        return None
    if kv_len.dtype == torch.bool:
        return pack_key_mask(kv_len.to(device))
    return kv_len.to(device=device, dtype=torch.int32).contiguous()


def flash_attention(q: torch.Tensor, k: torch.Tensor, v: torch.Tensor, causal: bool = False,
                    scale: float | None = None, kv_len: torch.Tensor | None = None,
                    alibi: torch.Tensor | None = None, window: int = 0, rowsum_col: int = -1,
                    max_col: int = -1) -> torch.Tensor:
    """softmax(scale * Q K^T + alibi + mask) V over [B, S, H, D] views.
    ``rowsum_col`` (inference): V's zero-padded column that the caller filled
    with ones -- the D=64 fast kernel then takes the softmax row sums from the
    output instead of summing on the VALU (the SD UNet's padded heads).
    ``max_col`` (inference, with ``rowsum_col``, 48-wide heads): K holds
    K * s * log2(e) with its zero-padded column ``max_col`` set to 1, where s is the
    true softmax scale, and ``scale`` must be ln 2 (attention_tiled.hip MC: the
    softmax offset rides in the S MFMA)."""
    scale = scale if scale is not None else 1.0 / math.sqrt(q.shape[-1])
    if alibi is not None:
        alibi = alibi.to(device=q.device, dtype=torch.float32).contiguous()
    if rowsum_col >= 0 and _lib.use_native(q, k, v) and not torch.is_grad_enabled():
        _check(q, k, v)
        return _fwd(q, k, v, causal, scale, native_mask(kv_len, q.device), alibi, window=window,
                    rowsum_col=rowsum_col, max_col=max_col)[0]
    if max_col >= 0:
        raise ValueError("max_col needs rowsum_col and the native inference path")
    if _lib.use_native(q, k, v):
        return _FlashAttnFn.apply(q, k, v, causal, scale, native_mask(kv_len, q.device), alibi, int(window))
    o, _ = attention_reference(q, k, v, causal, scale, kv_len, alibi, window)
    return o


def wide_head_attention(q: torch.Tensor, k: torch.Tensor, v: torch.Tensor, scale: float):
    """Single-head attention over [B, S, 512] bf16 rows (the VAE mid-block, inference) on the
    LDS-DMA flash kernel (attention_tiled.hip ``kca_attn_fwd_wide``). Returns None when the shape is
    outside that kernel, or when a row's softmax overflowed its first-tile reference max (one flag
    read back: the caller reruns those rare inputs on its GEMM path)."""
    if not (_lib.use_native(q, k, v) and q.dim() == 3 and q.shape[-1] == 512 and not torch.is_grad_enabled()):
        return None
    if any(t.stride(-1) != 1 or t.dtype != torch.bfloat16 for t in (q, k, v)):
        return None
    B, Sq, D = q.shape
    Sk = k.shape[1]
    if Sq % 128 or Sk % 32:
        return None
    o = torch.empty(B, Sq, D, device=q.device, dtype=q.dtype)
    flags = torch.empty(4 * (Sq // 128) * B, device=q.device, dtype=torch.int32)
    st = lambda t: (t.stride(0), t.stride(1), 0)  # noqa: E731  (one head: head stride unused)
    rc = _lib.call_rc("kca_attn_fwd_wide", q.data_ptr(), k.data_ptr(), v.data_ptr(), o.data_ptr(), None,
                      *st(q), *st(k), *st(v), *st(o), B, Sq, Sk, 1, 1, D, float(scale), flags.data_ptr(),
                      _lib.stream())
    if rc != 0 or bool(flags.any()):
        return None
    return o


class _QKVRopeAttnFn(torch.autograd.Function):
    """qkv: [B, S, 3*H*D] fused projection output (consumed and rotated in place)."""

    @staticmethod
    def forward(ctx, qkv, H, D, rot, interleaved, base, causal, scale, kv_len):
        B, S, _ = qkv.shape
        v5 = qkv.view(B, S, 3, H, D)
        q, k, v = v5[:, :, 0], v5[:, :, 1], v5[:, :, 2]
        if rot > 0:
            apply_rotary_(q, k, rot, S, interleaved, base, 1.0)
        o, lse = _fwd(q, k, v, causal, scale, kv_len, None)
        ctx.save_for_backward(qkv, o, lse, kv_len)
        ctx.cfg = (H, D, rot, interleaved, base, causal, scale)
        return o.view(B, S, H * D)

    @staticmethod
    def backward(ctx, do):
        qkv, o, lse, kv_len = ctx.saved_tensors
        H, D, rot, interleaved, base, causal, scale = ctx.cfg
        B, S, _ = qkv.shape
        v5 = qkv.view(B, S, 3, H, D)
        q, k, v = v5[:, :, 0], v5[:, :, 1], v5[:, :, 2]
        dqkv = torch.empty_like(qkv)
        d5 = dqkv.view(B, S, 3, H, D)
        dq, dk, dv = d5[:, :, 0], d5[:, :, 1], d5[:, :, 2]
        do = do.contiguous().view(B, S, H, D)
        _bwd(q, k, v, o, do, lse, dq, dk, dv, causal, scale, kv_len, None)
        if rot > 0:
            apply_rotary_(dq, dk, rot, S, interleaved, base, -1.0)
        return dqkv, None, None, None, None, None, None, None, None


def qkv_rope_attention(qkv: torch.Tensor, n_heads: int, head_dim: int, rot: int,
                       interleaved: bool, causal: bool = True, base: float = 10000.0,
                       scale: float | None = None,
                       kv_len: torch.Tensor | None = None) -> torch.Tensor:
    """Fused (RoPE + attention) over a [B, S, 3*H*D] QKV buffer -> [B, S, H*D]."""
    B, S, _ = qkv.shape
    scale = scale if scale is not None else 1.0 / math.sqrt(head_dim)
    if _lib.use_native(qkv):
        return _QKVRopeAttnFn.apply(qkv.contiguous(), n_heads, head_dim, rot, interleaved, base,
                                    causal, scale, native_mask(kv_len, qkv.device))
    v5 = qkv.view(B, S, 3, n_heads, head_dim)
    q, k, v = v5[:, :, 0], v5[:, :, 1], v5[:, :, 2]
    if rot > 0:
        q, k = _rope_out_of_place(q, k, rot, interleaved, base)
    o, _ = attention_reference(q, k, v, causal, scale, kv_len, None)
    return o.reshape(B, S, n_heads * head_dim)


def _rope_out_of_place(q, k, rot, interleaved, base):
    from .rope import rope_tables, _rotate_ref
    B, S = q.shape[:2]
    cos, sin = rope_tables(rot, S, base, q.device)
    pos = torch.arange(S, device=q.device).repeat(B)
    c, s = cos[pos], sin[pos]
    qo = _rotate_ref(q.reshape(B * S, *q.shape[2:]), c, s, interleaved, 1.0).view(q.shape)
    ko = _rotate_ref(k.reshape(B * S, *k.shape[2:]), c, s, interleaved, 1.0).view(k.shape)
    return qo, ko
