"""Decode-path ops (K11/K12/K13/K31/K32) for the serving engine.

* ``decode_prep``       RoPE on the step's Q/K + append K/V into the slot cache
* ``decode_attention``  split-K flash-decoding over the head-major slot cache
* ``sample_logits``     fused penalty/bans/temperature/top-k/top-p/multinomial

bf16 and fp16 GPU tensors run ``csrc/kernels/decode.hip`` (fp16: the ``*_f16`` entries); CPU tensors run the fp32
references below (same semantics; used by the CPU test-suite and to pin the
kernels in ``tests/test_decode_gpu.py``).

Cache layout: ``k_cache``/``v_cache`` are [slots, Hkv, max_len, D] (one per
layer); a request owns one slot for its lifetime. Paged (``block_table``
given): they are page pools [pages, Hkv, PS, D] (PS a power of two >= 16) and
token t of sequence ``slots[b]`` lives in page ``block_table[slots[b], t // PS]``
at row ``t % PS`` -- a request holds only the pages it has filled, and beams
share their common prefix pages (``engine.runner.KVCache``).
"""
from __future__ import annotations

import os

import math

import torch

from . import _lib


# ------------------------------------------------------------------- prep
def decode_prep(qkv: torch.Tensor, n_heads: int, kv_heads: int, head_dim: int, rot: int,
                interleaved: bool, cos: torch.Tensor | None, sin: torch.Tensor | None,
                pos: torch.Tensor, slots: torch.Tensor, k_cache: torch.Tensor, v_cache: torch.Tensor,
                block_table: torch.Tensor | None = None):
    """qkv: [B, (H+2Hkv)*D] (row-strided). Rotates Q in place, writes rotated K and
    V of each row b into cache[slots[b], :, pos[b]] (paged: into its page)."""
    B = qkv.shape[0]
    H, Hkv, D = n_heads, kv_heads, head_dim
    if _lib.use_native(qkv, k_cache):
        assert qkv.stride(-1) == 1 and k_cache.stride(-1) == 1 and k_cache.stride() == v_cache.stride()
        assert pos.dtype == torch.int32 and slots.dtype == torch.int32
        tbl, tstride, shift = _table_args(block_table, k_cache)
        _lib.call("kca_decode_prep", qkv.data_ptr(), qkv.stride(0), B, H, Hkv, D, rot, int(interleaved),
                  _lib.ptr(cos), _lib.ptr(sin), pos.data_ptr(), slots.data_ptr(), k_cache.data_ptr(),
                  v_cache.data_ptr(), k_cache.stride(0), k_cache.stride(1), k_cache.stride(2), tbl, tstride, shift,
                  _lib.stream())
        return
    rows = qkv.view(B, H + 2 * Hkv, D)
    x = rows.to(torch.float32, copy=True)  # never alias: K rows of qkv stay unrotated
    if rot > 0:
        half = rot // 2
        p = pos.long()
        c, s = cos[p][:, None, :], sin[p][:, None, :]  # [B, 1, rot/2]
        xr = x[:, :H + Hkv, :rot]
        if interleaved:
            a, b = xr[..., 0::2], xr[..., 1::2]
            out = torch.stack((a * c - b * s, b * c + a * s), dim=-1).flatten(-2)
        else:
            a, b = xr[..., :half], xr[..., half:]
            out = torch.cat((a * c - b * s, b * c + a * s), dim=-1)
        x[:, :H + Hkv, :rot] = out
        rows[:, :H, :rot] = x[:, :H, :rot].to(rows.dtype)
    sl, p = slots.long(), pos.long()
    if block_table is not None:
        PS = k_cache.shape[2]
        sl, p = block_table.long()[sl, p // PS], p % PS
    k_cache[sl, :, p] = x[:, H:H + Hkv].to(k_cache.dtype)
    v_cache[sl, :, p] = x[:, H + Hkv:].to(v_cache.dtype)


def _table_args(block_table, k_cache):
    """(pointer, row stride, log2 page size) of a paged cache's block table."""
    if block_table is None:
        return 0, 0, 0
    PS = k_cache.shape[2]
    assert PS >= 16 and PS & (PS - 1) == 0, "page size must be a power of two >= 16"
    assert block_table.dtype == torch.int32 and block_table.is_contiguous()
    return block_table.data_ptr(), block_table.stride(0), PS.bit_length() - 1


def gather_kv(cache: torch.Tensor, seq: int, n: int, block_table: torch.Tensor | None = None) -> torch.Tensor:
    """Tokens [0, n) of sequence ``seq`` as a [Hkv, n, D] tensor (contiguous or paged cache)."""
    if block_table is None:
        return cache[seq, :, :n]
    PS = cache.shape[2]
    pages = block_table[seq, :-(-n // PS)].long()
    Hkv, D = cache.shape[1], cache.shape[3]
    return cache[pages].transpose(0, 1).reshape(Hkv, -1, D)[:, :n]


# -------------------------------------------------------------- attention
def decode_ws_floats(B: int, H: int, Hkv: int, D: int, max_kv: int, chunk: int = 0) -> int:
    if chunk <= 0:
        chunk = decode_chunk(B, Hkv, max_kv)
    ns = -(-max_kv // chunk)
    # the first B*H words (padded to 16 B) are the split-K fan-in counters (csrc/kernels/decode.hip):
    # a workspace must be ZERO-initialised before its first use (the kernel re-arms them after)
    return -(-(B * H) // 4) * 4 + B * H * ns * (D + 2) if ns > 1 else 0


_DECODE_WGS = int(os.environ.get("KCA_DECODE_SPLIT_TARGET", "256"))  # split-K workgroup target (A/B knob)


def decode_chunk(B: int, Hkv: int, max_kv: int) -> int:
    """Mirror of kca_decode_chunk. Measured on MI355X with cold caches (the decode
    regime: a layer's KV was last touched a full weight stream ago;
    profiles/decode_attn_cold_sweep_r2.jsonl): a split of the one-pass kernel costs
    about one HBM round trip per 32 tokens, so ~256 (sequence, head, split)
    workgroups of >= 64 tokens beat many short splits (B=1, 600 cached tokens: 64-token
    splits 11.5 us vs 32-token 20.1 us), a cache of <= 256 tokens is one split, and
    long caches stop at 256-token splits (more workgroups beat longer chains there)."""
    if max_kv <= 256:
        return max(64, -(-max_kv // 32) * 32)
    work = B * Hkv
    want = -(-_DECODE_WGS // work)
    c = -(-max_kv // want)
    c = -(-c // 32) * 32
    cap = 256 if max_kv >= 2048 else 1024
    return max(64, min(cap, c))


def decode_attention(q: torch.Tensor, k_cache: torch.Tensor, v_cache: torch.Tensor, slots: torch.Tensor,
                     kv_lens: torch.Tensor, n_heads: int, max_kv: int, scale: float | None = None,
                     alibi: torch.Tensor | None = None, out: torch.Tensor | None = None,
                     ws: torch.Tensor | None = None, chunk: int = 0,
                     block_table: torch.Tensor | None = None, window: int = 0) -> torch.Tensor:
    """q: [B, >=H*D] (row-strided; e.g. the Q slice of the fused QKV buffer).
    Attends row b over cache[slots[b], :, :kv_lens[b]] (paged: over its pages),
    or over its last ``window`` positions (GPT-Neo local layers). Returns [B, H*D]."""
    B = q.shape[0]
    _, Hkv, L, D = k_cache.shape
    H = n_heads
    scale = scale if scale is not None else 1.0 / math.sqrt(D)
    if out is None:
        out = torch.empty(B, H * D, device=q.device, dtype=q.dtype)
    if _lib.use_native(q, k_cache):
        assert q.stride(-1) == 1 and out.stride(-1) == 1 and k_cache.stride() == v_cache.stride()
        tbl, tstride, shift = _table_args(block_table, k_cache)
        assert max_kv <= (L if block_table is None else block_table.shape[1] * L)
        if chunk <= 0:
            chunk = decode_chunk(B, Hkv, max_kv)
        need = decode_ws_floats(B, H, Hkv, D, max_kv, chunk)
        if need and (ws is None or ws.numel() < need):
            ws = torch.zeros(need, device=q.device, dtype=torch.float32)
        _lib.call("kca_decode_attn", q.data_ptr(), q.stride(0), k_cache.data_ptr(), v_cache.data_ptr(),
                  k_cache.stride(0), k_cache.stride(1), k_cache.stride(2), slots.data_ptr(),
                  kv_lens.data_ptr(), out.data_ptr(), out.stride(0), _lib.ptr(ws),
                  ws.numel() if ws is not None else 0, B, H, Hkv, D, max_kv, chunk, float(scale),
                  _lib.ptr(alibi), tbl, tstride, shift, int(window), _lib.stream())
        return out
    return decode_attention_reference(q, k_cache, v_cache, slots, kv_lens, H, scale, alibi, out, block_table,
                                      window)


def decode_prep_attention(qkv: torch.Tensor, n_heads: int, kv_heads: int, head_dim: int, rot: int,
                          interleaved: bool, cos: torch.Tensor | None, sin: torch.Tensor | None,
                          pos: torch.Tensor, slots: torch.Tensor, k_cache: torch.Tensor, v_cache: torch.Tensor,
                          kv_lens: torch.Tensor, max_kv: int, scale: float | None = None,
                          alibi: torch.Tensor | None = None, out: torch.Tensor | None = None,
                          ws: torch.Tensor | None = None, block_table: torch.Tensor | None = None,
                          window: int = 0, by_row: int = 0) -> torch.Tensor:
    """``decode_prep`` + ``decode_attention`` for the decode step (kv_lens = pos + 1).
    ``by_row``: per-step descriptors as in ``decode_prep_attention_gemv`` (native path only).
    Native: ONE launch (``kca_decode_prep_attn``) that rotates Q itself and lets
    the split holding the new token rotate and append K/V (the prep kernel's ~5 us
    per layer at B=1 disappears); bit-identical to the two-kernel path."""
    B = qkv.shape[0]
    _, Hkv, L, D = k_cache.shape
    H = n_heads
    scale = scale if scale is not None else 1.0 / math.sqrt(D)
    f16 = qkv.is_cuda and qkv.dtype == torch.float16 and k_cache.dtype == torch.float16
    if (_lib.use_native(qkv, k_cache) and _lib.has("kca_decode_prep_attn")) or (f16 and _lib.has("kca_decode_prep_attn_f16")):
        assert qkv.stride(-1) == 1 and k_cache.stride() == v_cache.stride()
        assert kv_lens.dtype == torch.int32 and slots.dtype == torch.int32
        if out is None:
            out = torch.empty(B, H * D, device=qkv.device, dtype=qkv.dtype)
        tbl, tstride, shift = _table_args(block_table, k_cache)
        chunk = decode_chunk(B, Hkv, max_kv)
        need = decode_ws_floats(B, H, Hkv, D, max_kv, chunk)
        if need and (ws is None or ws.numel() < need):
            ws = torch.zeros(need, device=qkv.device, dtype=torch.float32)
        _lib.call("kca_decode_prep_attn_f16" if f16 else "kca_decode_prep_attn", qkv.data_ptr(), qkv.stride(0),
                  k_cache.data_ptr(), v_cache.data_ptr(),
                  k_cache.stride(0), k_cache.stride(1), k_cache.stride(2), slots.data_ptr(), kv_lens.data_ptr(),
                  out.data_ptr(), out.stride(0), _lib.ptr(ws), ws.numel() if ws is not None else 0, B, H, Hkv, D,
                  max_kv, chunk, float(scale), _lib.ptr(alibi), tbl, tstride, shift, rot, int(interleaved),
                  _lib.ptr(cos), _lib.ptr(sin), int(window), int(by_row), _lib.stream())
        return out
    assert not by_row, "per-step descriptors are a native-kernel feature"
    decode_prep(qkv, H, Hkv, D, rot, interleaved, cos, sin, pos, slots, k_cache, v_cache, block_table)
    return decode_attention(qkv, k_cache, v_cache, slots, kv_lens, H, max_kv, scale, alibi, out, ws,
                            block_table=block_table, window=window)


def decode_prep_attention_gemv(qkv, n_heads, kv_heads, head_dim, rot, interleaved, cos, sin, pos, slots,
                               k_cache, v_cache, kv_lens, max_kv, scale, alibi, out, ws, block_table, window,
                               gx: torch.Tensor, gw: torch.Tensor, gbias: torch.Tensor | None, gy: torch.Tensor,
                               act: int, by_row: int = 0) -> bool:
    """Fused decode layer, part 1 (batch 1; csrc/kernels/decode.hip decode_attn_gemv_kernel): the
    ``decode_prep_attention`` launch and the fc_in GEMV ``gy = act(gx W^T + b)`` as ONE launch
    (attention workgroups first, the weight stream on the rest). Returns False (nothing launched)
    for shapes outside the fused variants; the caller then runs the two separately.
    ``by_row``: bit 0 -- ``cos`` / ``sin`` are the step's rows (row b = sequence b's angles at its
    position), bit 1 -- ``block_table`` row b is sequence b's page row (per-step descriptors uploaded
    with the step's inputs: the attention chain does not wait for the length or the slot first)."""
    B = qkv.shape[0]
    _, Hkv, L, D = k_cache.shape
    f16 = _lib.native_f16(qkv, k_cache, gx, gw)
    if not ((_lib.use_native(qkv, k_cache, gx, gw) or f16) and _lib.has("kca_decode_prep_attn_gemv") and B == 1
            and gx.is_contiguous() and gw.is_contiguous() and gy.is_contiguous()
            and (gbias is None or gbias.dtype == gx.dtype)):
        return False
    tbl, tstride, shift = _table_args(block_table, k_cache)
    chunk = decode_chunk(B, Hkv, max_kv)
    need = decode_ws_floats(B, n_heads, Hkv, D, max_kv, chunk)
    if need and (ws is None or ws.numel() < need):
        return False
    fn = getattr(_lib.require(), "kca_decode_prep_attn_gemv_f16" if f16 else "kca_decode_prep_attn_gemv")
    rc = fn(
        qkv.data_ptr(), qkv.stride(0), k_cache.data_ptr(), v_cache.data_ptr(), k_cache.stride(0), k_cache.stride(1),
        k_cache.stride(2), slots.data_ptr(), kv_lens.data_ptr(), out.data_ptr(), out.stride(0), _lib.ptr(ws),
        ws.numel() if ws is not None else 0, B, n_heads, Hkv, D, max_kv, chunk, float(scale), _lib.ptr(alibi), tbl,
        tstride, shift, rot, int(interleaved), _lib.ptr(cos), _lib.ptr(sin), int(window), gx.data_ptr(),
        gw.data_ptr(), _lib.ptr(gbias), gy.data_ptr(), gw.shape[0], gw.shape[1], int(act), int(by_row), _lib.stream())
    if rc == 10:
        return False
    if rc != 0:
        raise RuntimeError(f"kca_decode_prep_attn_gemv returned status {rc}")
    _lib.LAUNCHES[0] += 1
    return True


def gemv_dual_ln(x1: torch.Tensor, w1: torch.Tensor, x2: torch.Tensor | None, w2: torch.Tensor | None, bias,
                 h: torch.Tensor, gamma: torch.Tensor, beta, eps: float, ypart: torch.Tensor, cnt: torch.Tensor,
                 h_out: torch.Tensor, xn_out: torch.Tensor, gamma2: torch.Tensor | None = None, beta2=None,
                 xn2_out: torch.Tensor | None = None) -> None:
    """Fused decode layer, tail (batch 1; ``kca_gemv_dual_ln``): y = x1 W1^T (+ x2 W2^T) + b, then
    h_out = h + y and xn_out = LayerNorm(h_out) in one launch -- GPT-J's out-projection + fc_out +
    parallel residual (two weight streams), a sequential-residual layer's out-projection or fc_out
    (``x2`` None), and with ``gamma2`` the second LayerNorm of the same h_out into ``xn2_out`` (GPT-NeoX:
    ln_1 and ln_2 of one residual stream share the statistics). ``ypart``: >= N fp32 words;
    ``cnt``: zero-initialised int32 [32 * 65] arrival counters. N <= 16384."""
    _lib.call("kca_gemv_dual_ln_f16" if x1.dtype == torch.float16 else "kca_gemv_dual_ln", x1.data_ptr(), w1.data_ptr(), w1.shape[1], _lib.ptr(x2), _lib.ptr(w2),
              w2.shape[1] if w2 is not None else 0, _lib.ptr(bias), ypart.data_ptr(), cnt.data_ptr(), h.data_ptr(),
              h_out.data_ptr(), gamma.data_ptr(), _lib.ptr(beta), float(eps), xn_out.data_ptr(), _lib.ptr(gamma2),
              _lib.ptr(beta2), _lib.ptr(xn2_out), w1.shape[0], _lib.stream())


def gemv_dual_ln_reference(x1, w1, x2, w2, bias, h, gamma, beta, eps):
    """fp32 reference of ``gemv_dual_ln``: (h + y rounded to bf16, LayerNorm of it)."""
    y = x1.float() @ w1.float().t()
    if x2 is not None:
        y = y + x2.float() @ w2.float().t()
    if bias is not None:
        y = y + bias.float()
    hn = (h.float() + y).to(h.dtype)
    xn = torch.nn.functional.layer_norm(hn.float(), (hn.shape[-1],), gamma.float(),
                                        beta.float() if beta is not None else None, eps)
    return hn, xn


def decode_attention_reference(q, k_cache, v_cache, slots, kv_lens, n_heads, scale, alibi=None, out=None,
                               block_table=None, window: int = 0):
    B = q.shape[0]
    _, Hkv, L, D = k_cache.shape
    H = n_heads
    if out is None:
        out = torch.empty(B, H * D, device=q.device, dtype=q.dtype)
    for b in range(B):
        n = int(kv_lens[b])
        lo = max(0, n - window) if window > 0 else 0
        s_ = int(slots[b])
        qb = q[b, :H * D].float().view(H, D)
        kb = gather_kv(k_cache, s_, n, block_table)[:, lo:].float().repeat_interleave(H // Hkv, 0)  # [H, n, D]
        vb = gather_kv(v_cache, s_, n, block_table)[:, lo:].float().repeat_interleave(H // Hkv, 0)
        sc = torch.einsum("hd,hnd->hn", qb, kb) * scale
        if alibi is not None:
            sc = sc + alibi.float()[:, None] * (torch.arange(lo, n, device=q.device) - (n - 1)).float()[None]
        o = torch.einsum("hn,hnd->hd", sc.softmax(-1), vb)
        out[b] = o.reshape(-1).to(out.dtype)
    return out


# --------------------------------------------------------------- sampling
_CNT: dict = {}


def _sample_counters(dev: torch.device, B: int):
    """Zeroed per-row arrival counters of the multi-workgroup sampler (decode.hip sample_mwg_kernel
    re-arms them). Allocated outside graph capture (the runner warms up eagerly first); None inside
    a capture that would need a new buffer, which keeps those rows on the one-workgroup kernels."""
    c = _CNT.get(dev)
    if c is None or c.numel() < B:
        if torch.cuda.is_current_stream_capturing():
            return None
        c = _CNT[dev] = torch.zeros(max(4096, B), dtype=torch.int32, device=dev)
    return c


def sample_logits(logits: torch.Tensor, *, temperature: torch.Tensor, top_k: torch.Tensor,
                  top_p: torch.Tensor, rep_penalty: torch.Tensor | None = None,
                  seen: torch.Tensor | None = None, slots: torch.Tensor | None = None,
                  ban_ids: torch.Tensor | None = None, seeds: torch.Tensor | None = None, step: int = 0,
                  ws: torch.Tensor | None = None, out_ids: torch.Tensor | None = None,
                  out_logprobs: torch.Tensor | None = None, out_kept: torch.Tensor | None = None,
                  mwg_complete: bool = False):
    """Per-row parameters (all [B]): temperature (<= 0 -> greedy), top_k (0 = off),
    top_p (1 = off), rep_penalty. ``seen`` is a [slots, V] uint8 mask of tokens
    already in each sequence (repetition penalty; the chosen id is marked).
    ``ban_ids`` [B, n] (-1 padded) get -inf. Returns (ids int64 [B], logprob [B])
    where logprob is under the penalised, temperature-scaled distribution.
    ``mwg_complete``: the caller guarantees every row is greedy or has 1 <= top_k <= MWG_KMAX
    (``mwg_complete_rows``), so the multi-workgroup kernel finishes every row and the closing
    one-workgroup kernel is not launched."""
    B, V = logits.shape
    dev = logits.device
    if out_ids is None:
        out_ids = torch.empty(B, dtype=torch.int64, device=dev)
    if out_logprobs is None:
        out_logprobs = torch.empty(B, dtype=torch.float32, device=dev)
    if logits.is_cuda and logits.dtype in (torch.bfloat16, torch.float32, torch.float16):
        if ws is None or ws.numel() < B * V:
            ws = torch.empty(B * V, device=dev, dtype=torch.float32)
        assert logits.stride(-1) == 1
        n_ban = ban_ids.shape[1] if ban_ids is not None else 0
        cnt = _sample_counters(dev, B)
        _lib.call("kca_sample_logits", logits.data_ptr(), logits.stride(0),
                  {torch.float32: 0, torch.bfloat16: 1, torch.float16: 2}[logits.dtype], B, V,
                  temperature.data_ptr(), top_k.data_ptr(),
                  top_p.data_ptr(), _lib.ptr(rep_penalty), _lib.ptr(seen), _lib.ptr(slots),
                  _lib.ptr(ban_ids), n_ban, _lib.ptr(seeds), int(step), ws.data_ptr(),
                  out_ids.data_ptr(), out_logprobs.data_ptr(), _lib.ptr(out_kept), _lib.ptr(cnt),
                  int(bool(mwg_complete)), _lib.stream())
        return out_ids, out_logprobs
    return sample_logits_reference(logits, temperature, top_k, top_p, rep_penalty, seen, slots, ban_ids,
                                   seeds, step, out_ids, out_logprobs, out_kept)


MWG_KMAX = 64  # decode.hip: top-k rows the multi-workgroup sampler takes


def mwg_complete_rows(temperatures, top_ks) -> bool:
    """Host-side check for ``sample_logits(mwg_complete=True)``: every row greedy or 1 <= top_k <= 64."""
    return all((not t > 0) or 1 <= int(k) <= MWG_KMAX for t, k in zip(temperatures, top_ks))


def processed_logits_reference(logits, temperature, rep_penalty, seen, slots, ban_ids):
    x = logits.float().clone()
    B, V = x.shape
    for b in range(B):
        slot = int(slots[b]) if slots is not None else b
        rp = float(rep_penalty[b]) if rep_penalty is not None else 1.0
        if rp != 1.0 and seen is not None:
            m = seen[slot].bool()
            v = x[b, m]
            x[b, m] = torch.where(v < 0, v * rp, v / rp)
        if ban_ids is not None:
            ids = ban_ids[b][(ban_ids[b] >= 0) & (ban_ids[b] < V)].long()
            x[b, ids] = float("-inf")
        t = float(temperature[b])
        if t > 0 and t != 1.0:
            x[b] = x[b] / t
    return x


def keep_mask_reference(x: torch.Tensor, top_k: int, top_p: float) -> torch.Tensor:
    """HF TopK then TopP warper keep-mask for one row of processed logits."""
    keep = torch.isfinite(x)
    V = x.shape[0]
    if 0 < top_k < V:
        kth = torch.topk(x, top_k).values[-1]
        keep &= x >= kth
    if top_p < 1.0:
        xm = x.masked_fill(~keep, float("-inf"))
        srt, idx = torch.sort(xm, descending=False)
        cum = srt.softmax(-1).cumsum(-1)
        remove = cum <= (1 - top_p)
        remove[-1:] = False
        rm = torch.zeros_like(keep)
        rm[idx] = remove
        keep &= ~rm
    return keep


def sample_logits_reference(logits, temperature, top_k, top_p, rep_penalty=None, seen=None, slots=None,
                            ban_ids=None, seeds=None, step=0, out_ids=None, out_logprobs=None,
                            out_kept=None):
    B, V = logits.shape
    x = processed_logits_reference(logits, temperature, rep_penalty, seen, slots, ban_ids)
    lsm = torch.log_softmax(x, -1)
    ids = torch.empty(B, dtype=torch.int64, device=logits.device) if out_ids is None else out_ids
    lps = torch.empty(B, device=logits.device) if out_logprobs is None else out_logprobs
    for b in range(B):
        t = float(temperature[b])
        if not t > 0:
            i = int(torch.argmax(x[b]))
            kept = 1
        else:
            keep = keep_mask_reference(x[b], int(top_k[b]), float(top_p[b]))
            probs = torch.softmax(x[b].masked_fill(~keep, float("-inf")), -1)
            g = torch.Generator(device="cpu")
            g.manual_seed(((int(seeds[b]) if seeds is not None else b) * 1000003 + int(step)) % (1 << 63))
            i = int(torch.multinomial(probs.cpu(), 1, generator=g))
            kept = int(keep.sum())
        ids[b] = i
        lps[b] = lsm[b, i]
        if out_kept is not None:
            out_kept[b] = kept
        if seen is not None:
            seen[int(slots[b]) if slots is not None else b, i] = 1
    return ids, lps


__all__ = ["decode_prep", "decode_attention", "decode_prep_attention", "decode_attention_reference", "decode_chunk", "gather_kv",
           "decode_ws_floats", "sample_logits", "sample_logits_reference", "keep_mask_reference",
           "processed_logits_reference"]
