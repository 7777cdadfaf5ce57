"""Model runner for serving: slot KV cache, prefill, fused decode step, HIP graphs.

The FT-equivalent decode loop for every causal LM in
``models.causal_lm`` (GPT-2, GPT-J, GPT-NeoX/Pythia, GPT-Neo, BLOOM):

* ``KVCache``: paged by default -- per layer a pool of [Hkv, 64, D] pages and a
  block table per sequence slot (head-major pages, so each (sequence, head,
  page) is a contiguous HBM stream); ``page_size=0`` gives one contiguous
  [Hkv, max_len, D] slot per sequence. 288 GB of HBM holds e.g. 64 GPT-J
  sequences x 2048 tokens (60 GB) next to the 12 GB of weights; with pages, the
  slot count is no longer tied to that worst case.
* ``prefill``: prompts (ragged: right-padded in one batch) through the
  flash-attention kernel, K/V (post-RoPE) written into each sequence's pages.
* ``decode``: one token per running sequence -- fused QKV GEMM ->
  ``kca_decode_prep`` (RoPE + cache append) -> ``kca_decode_attn`` (split-K) ->
  out-proj, residual adds fused into the next LayerNorm -> LM head ->
  ``kca_sample_logits``. On GPU the whole step (all layers + sampling) is
  captured once per (batch bucket, kv bucket) into a HIP graph and replayed, so
  a GPT-J step is one graph launch + one 8-byte/row D2H copy.

Host inputs of a step (tokens, positions, slots, sampling params, bans, seeds)
travel in ONE packed pinned buffer -> one H2D copy. ``decode_async`` launches a
step without waiting for it and can take each row's input token from the
previous launch's device output, so the engine launches step t+1 before it
reads step t's tokens (``LLMEngine``'s one-step lookahead).
"""
from __future__ import annotations

import math
import os

import torch

from .. import ops
from ..ops import decode as dops
from ..ops import _lib
from ..ops import skinny_mm as smm
from ..ops.gemv import embed_ln_rows, ln_rows, ln_skinny_linear, skinny_linear

# decode steps: each row's RoPE angles and page-table row travel with the step's packed inputs (fixed
# device addresses), so every layer's attention chain loads them in its first memory round trip
# instead of after the length / slot arrive; KCA_DECODE_STEP_DESC=0: look them up on the device
_STEP_DESC = os.environ.get("KCA_DECODE_STEP_DESC", "1") not in ("0", "false")
# ... also for batch > 1 (the unfused per-layer path); KCA_DECODE_STEP_DESC_BATCHED=0: batch 1 only
_STEP_DESC_BATCHED = os.environ.get("KCA_DECODE_STEP_DESC_BATCHED", "1") not in ("0", "false")


def _next_pow2(n: int, lo: int = 1) -> int:
    p = lo
    while p < n:
        p *= 2
    return p


class KVCacheFull(RuntimeError):
    """No free KV page for a sequence (the engine's admission control keeps
    running requests clear of this)."""


class KVCache:
    """Per-layer K and V storage for the serving engine.

    ``page_size == 0``: contiguous slots [slots+1, Hkv, max_len, D] (a slot is
    one sequence's whole capacity). ``page_size > 0`` (default): paged pools
    [pages+1, Hkv, PS, D] plus a block table [slots+1, max_len/PS] (int32,
    device; host twin ``table_h``) -- a sequence holds only the pages it has
    filled, finished requests return theirs at once, and beams share their
    prefix pages (refcounted, ``fork`` copies only a partial tail page). The
    last page and the last table row are scratch: free table entries point at
    the scratch page, so a stray read or a graph bucket's padding row touches
    nothing live. Head-major pages keep each (sequence, head, page) a
    contiguous PS*D*2-byte stream for the decode kernel (``ops.decode``).
    """

    def __init__(self, n_layers: int, slots: int, kv_heads: int, max_len: int, head_dim: int,
                 device, dtype=torch.bfloat16, page_size: int = 0, n_pages: int | None = None,
                 layer_devices: list | None = None):
        self.slots, self.max_len, self.scratch = slots, max_len, slots
        self.page_size = page_size
        self.device = torch.device(device)
        # layer-split models (parallel.layer_split): each layer's cache lives on that layer's device
        self.layer_devices = [torch.device(d) for d in layer_devices] if layer_devices else [self.device] * n_layers
        self.devices = list(dict.fromkeys([self.device] + self.layer_devices))
        if page_size:
            if page_size < 16 or page_size & (page_size - 1):
                raise ValueError(f"page_size {page_size}: need a power of two >= 16")
            self.blocks = -(-max_len // page_size)
            # default: every slot can hold a full-length sequence, plus one page per slot of headroom
            # for beam forks (a fork copies a partial tail page before the old one is dropped)
            self.n_pages = int(n_pages or slots * (self.blocks + 1))
            self.scratch_page = self.n_pages
            shape = (self.n_pages + 1, kv_heads, page_size, head_dim)
            self.table_h = torch.full((slots + 1, self.blocks), self.n_pages, dtype=torch.int32)
            self.tables = {d: self.table_h.to(d) for d in self.devices}
            self.table = self.tables[self.device]
            self.free_pages = list(range(self.n_pages - 1, -1, -1))
            self.ref = [0] * self.n_pages
            self.pages: list[list[int]] = [[] for _ in range(slots + 1)]
            self._dirty = False
        else:
            self.table = None
            self.n_pages = 0
            shape = (slots + 1, kv_heads, max_len, head_dim)
            self.tables = {}
        self.k = [torch.zeros(shape, device=d, dtype=dtype) for d in self.layer_devices]
        self.v = [torch.zeros(shape, device=d, dtype=dtype) for d in self.layer_devices]

    def nbytes(self) -> int:
        return sum(t.numel() * t.element_size() for t in self.k + self.v)

    @property
    def paged(self) -> bool:
        return self.page_size > 0

    def pages_for(self, n_tokens: int) -> int:
        return -(-n_tokens // self.page_size) if self.paged else 0

    def free_count(self) -> int:
        return len(self.free_pages) if self.paged else 0

    # ------------------------------------------------------------ page table
    def reserve(self, slot: int, n_tokens: int):
        """Make positions [0, n_tokens) of ``slot`` addressable (allocates pages)."""
        if not self.paged:
            return
        own = self.pages[slot]
        need = self.pages_for(min(n_tokens, self.max_len)) - len(own)
        if need <= 0:
            return
        if need > len(self.free_pages):
            raise KVCacheFull(f"slot {slot} needs {need} KV pages, {len(self.free_pages)} free")
        for _ in range(need):
            pg = self.free_pages.pop()
            self.ref[pg] = 1
            self.table_h[slot, len(own)] = pg
            own.append(pg)
        self._dirty = True

    def _drop(self, pages):
        for pg in pages:
            self.ref[pg] -= 1
            if self.ref[pg] == 0:
                self.free_pages.append(pg)

    def release(self, slot: int):
        if not self.paged or not self.pages[slot]:
            return
        self._drop(self.pages[slot])
        self.pages[slot] = []
        self.table_h[slot].fill_(self.scratch_page)
        self._dirty = True

    def sync(self):
        """Block-table edits -> device (stream-ordered after the work already queued)."""
        if self.paged and self._dirty:
            for t in self.tables.values():
                t.copy_(self.table_h)
            self._dirty = False

    def table_on(self, dev):
        return self.tables.get(torch.device(dev)) if self.paged else None

    def _per_layer(self, idx: list[int]):
        """``idx`` as a long tensor on every cache device."""
        t = torch.tensor(idx, dtype=torch.long)
        return {d: t.to(d) for d in self.devices}

    def fork(self, dst: list[int], src: list[int], upto: int):
        """Sequence ``src[i]`` positions [0, upto) -> ``dst[i]``. Paged: whole
        pages are shared (refcount), only a partial last page is copied; a
        permutation (dst and src overlapping) is safe."""
        if not dst:
            return
        if not self.paged:
            d, s = self._per_layer(dst), self._per_layer(src)
            for k, v, dev in zip(self.k, self.v, self.layer_devices):
                k[d[dev], :, :upto] = k[s[dev], :, :upto]  # RHS gathered first: overlapping permutations are safe
                v[d[dev], :, :upto] = v[s[dev], :, :upto]
            return
        full, part = divmod(upto, self.page_size)
        new_lists, cp_from, cp_to = [], [], []
        for d_, s_ in zip(dst, src):
            shared = self.pages[s_][:full]
            for pg in shared:
                self.ref[pg] += 1
            lst = list(shared)
            if part:
                if not self.free_pages:
                    self._drop([pg for l_ in new_lists for pg in l_] + lst)
                    raise KVCacheFull("no free KV page for a beam fork")
                pg = self.free_pages.pop()
                self.ref[pg] = 1
                cp_from.append(self.pages[s_][full])
                cp_to.append(pg)
                lst.append(pg)
            new_lists.append(lst)
        if cp_to:
            a, b = self._per_layer(cp_from), self._per_layer(cp_to)
            for k, v, dev in zip(self.k, self.v, self.layer_devices):
                k[b[dev]] = k[a[dev]]
                v[b[dev]] = v[a[dev]]
        for d_, lst in zip(dst, new_lists):  # old dst pages go only after every source was read
            self._drop(self.pages[d_])
            self.pages[d_] = lst
            self.table_h[d_].fill_(self.scratch_page)
            if lst:
                self.table_h[d_, :len(lst)] = torch.tensor(lst, dtype=torch.int32)
        self._dirty = True

    # --------------------------------------------------------------- prefill
    def plan_write(self, slots: list[int], lens: list[int], T: int, start: list[int] | None = None):
        """Index plan for writing prompts (right-padded to T) into the cache;
        ``start``: first position of each row (chunked prefill continues a slot)."""
        if not self.paged:
            return None
        import numpy as np
        PS = self.page_size
        start = start or [0] * len(slots)
        pg, off, src = [], [], []
        for i, (s_, L, p0) in enumerate(zip(slots, lens, start)):
            t = np.arange(p0, p0 + L)
            own = np.asarray(self.pages[s_][:self.pages_for(p0 + L)], dtype=np.int64)
            pg.append(own[t // PS])
            off.append(t % PS)
            src.append(i * T + t - p0)
        host = [torch.from_numpy(np.concatenate(xs)) for xs in (pg, off, src)]
        return {d: tuple(t.to(d) for t in host) for d in self.devices}

    def write(self, li: int, k: torch.Tensor, v: torch.Tensor, slots: list[int], lens: list[int], plan,
              start: list[int] | None = None):
        """k, v: [n, T, Hkv, D] (strided views of the QKV GEMM output)."""
        kc, vc = self.k[li], self.v[li]
        if plan is None:
            start = start or [0] * len(slots)
            for i, (s_, L, p0) in enumerate(zip(slots, lens, start)):  # strided copies (index scatter is ~4x slower)
                kc[s_, :, p0:p0 + L].copy_(k[i, :L].transpose(0, 1))
                vc[s_, :, p0:p0 + L].copy_(v[i, :L].transpose(0, 1))
            return
        pg, off, src = plan[self.layer_devices[li]]
        n, T, Hkv, D = k.shape
        kc[pg, :, off] = k.reshape(n * T, Hkv, D)[src]
        vc[pg, :, off] = v.reshape(n * T, Hkv, D)[src]


class _Packed:
    """Several small typed arrays in one byte buffer: two pinned host buffers
    (alternating per launch, so the host fills one while the previous launch's
    H2D copy may still be pending) + one device twin the decode graph reads."""

    def __init__(self, fields, device):
        self.off, self.fields = {}, fields
        o = 0
        for name, (dt, n) in fields.items():
            o = (o + 7) // 8 * 8
            self.off[name] = o
            o += n * torch.empty(0, dtype=dt).element_size()
        self.nbytes = (o + 7) // 8 * 8
        pin = device.type == "cuda"
        self.hosts = [torch.zeros(self.nbytes, dtype=torch.uint8, pin_memory=pin) for _ in range(2)]
        self.dev = torch.zeros(self.nbytes, dtype=torch.uint8, device=device)
        # numpy views of the pinned host buffers: per-row scalar writes cost
        # ~0.1 us instead of a torch indexing op (~5 us) each
        self._nps = [{name: self._view(h, name).numpy() for name in fields} for h in self.hosts]
        self.cur = 0

    def flip(self):
        self.cur ^= 1

    @property
    def host(self):
        return self.hosts[self.cur]

    @property
    def np(self):
        return self._nps[self.cur]

    def _view(self, buf, name):
        dt, n = self.fields[name]
        o = self.off[name]
        es = torch.empty(0, dtype=dt).element_size()
        return buf[o:o + n * es].view(dt)

    def h(self, name):
        return self._view(self.host, name)

    def d(self, name):
        return self._view(self.dev, name)

    def upload(self):
        self.dev.copy_(self.host, non_blocking=True)


class DecodeHandle:
    """A launched decode step: its sampled ids / log-probs land in pinned host
    memory behind an event; ``result()`` waits for them. ``ids_dev`` is the
    device output the next launch may chain its input tokens from."""

    __slots__ = ("ids_h", "lps_h", "n", "event", "ids_dev", "_res")

    def __init__(self, ids_h, lps_h, n, event, ids_dev):
        self.ids_h, self.lps_h, self.n, self.event, self.ids_dev = ids_h, lps_h, n, event, ids_dev
        self._res = None

    def result(self):
        if self._res is None:
            if self.event is not None:
                self.event.synchronize()
            self._res = (self.ids_h[:self.n].tolist(), self.lps_h[:self.n].tolist())
        return self._res


class ModelRunner:
    def __init__(self, model, max_slots: int = 32, max_len: int | None = None, use_graphs: bool | None = None,
                 max_bans: int = 16, page_size: int | None = None, kv_pages: int | None = None):
        self.model = model.eval()
        cfg = model.cfg
        self.cfg = cfg
        p = next(model.parameters())
        self.device, self.dtype = p.device, p.dtype
        self.max_len = max_len or cfg.max_pos
        # local heads: a tensor-parallel shard holds H/tp of them (parallel.tensor_parallel)
        self.H = model.h[0].attn.n_heads
        self.Hkv = self.H * cfg.kv_heads // cfg.n_heads
        self.D = cfg.head_dim
        self.V = cfg.vocab_size
        if page_size is None:
            page_size = int(os.environ.get("KCA_KV_PAGE_SIZE", "64"))
        # layer-split placement (parallel.layer_split): per-layer devices, the head's device
        self.layer_devs = [blk.ln_1.weight.device for blk in model.h]
        self.head_dev = model.ln_f.weight.device
        self.multi_device = len({str(d) for d in self.layer_devs + [self.device, self.head_dev]}) > 1
        self.cache = KVCache(cfg.n_layers, max_slots, self.Hkv, self.max_len, self.D, self.device, self.dtype,
                             page_size=page_size, n_pages=kv_pages, layer_devices=self.layer_devs)
        self.max_slots = max_slots
        self.rot = cfg.rotary_dim
        self._rope = {}
        for d in self.cache.devices:
            self._rope[d] = ops.rope_tables(self.rot, self.max_len, cfg.rotary_base, d) if self.rot > 0 else (None, None)
        self.cos, self.sin = self._rope[self.device]
        self._rope_h = (self.cos.cpu().numpy(), self.sin.cpu().numpy()) if self.rot > 0 else None
        self._step_desc = None
        self.seen = torch.zeros(max_slots + 1, self.V, dtype=torch.uint8, device=self.device)
        self.max_bans = max_bans
        on_gpu = self.device.type == "cuda"
        if on_gpu:  # MI355X-tuned hipBLASLt/rocBLAS choices for the batched decode GEMMs (utils/tunable.py)
            from ..utils import tunable
            tunable.ensure(tunable.DECODE_FILE)
        self.use_graphs = on_gpu if use_graphs is None else (use_graphs and on_gpu)
        if self.multi_device:
            self.use_graphs = False  # one graph cannot span devices; the split path runs eagerly
        self._graphs: dict = {}
        self._pool = None
        self._static: dict = {}
        # parallel-residual models (GPT-J, NeoX): the MLP branch does not depend on attention, so at
        # decode its two weight-streaming GEMVs run on a side stream while the latency-bound attention
        # chain (split-K attention, combine, out-proj) runs on the main one -- both captured into the
        # step's graph as a fork/join. Not under TP: two concurrent collectives could interleave
        # differently across ranks.
        from ..parallel.tensor_parallel import RowParallelLinear
        from ..parallel.tp_emulation import is_emulated
        rows = [mm for mm in model.modules() if isinstance(mm, RowParallelLinear)]
        tp = bool(rows)
        # one rank of a TP layout on one GPU (parallel/tp_emulation.py): its collectives are local
        # stand-ins, so the fused single-device layer applies to its shard shapes
        tp_local = all(is_emulated(mm.group) for mm in rows)
        self._par_mlp = (cfg.parallel_residual and on_gpu and not tp and not self.multi_device
                         and os.environ.get("KCA_DECODE_PAR_MLP", "1") not in ("0", "false"))
        self._side = torch.cuda.Stream(device=self.device) if self._par_mlp else None
        # batch-1 decode layer on ONE queue, the residual add and the next LayerNorm in the tail of the
        # projection that produces it (ops/decode.py gemv_dual_ln), no LayerNorm launch of its own:
        #   "gptj" parallel residual, one shared LN: QKV GEMV -> attention + fc_in -> out + fc_out + LN
        #   "neox" parallel residual, ln_1 / ln_2 of the same h: as gptj, the tail writes both norms
        #   "seq"  sequential residual (BLOOM, GPT-2, GPT-Neo): QKV GEMV -> attention -> out-proj +
        #          residual + ln_2 -> fc_in GEMV -> fc_out + residual + next ln_1
        # KCA_DECODE_FUSED=0: the per-projection path (two-stream for parallel-residual models)
        ln2 = [blk.ln_2 for blk in model.h]
        self._layer_kind = ("gptj" if all(x is None for x in ln2) else "neox") if cfg.parallel_residual else "seq"
        # a real TP group (BLOOM TP=8 serving): sequential layers close each row-parallel projection with
        # the custom all-reduce's fused residual + LayerNorm tail (parallel/custom_ar.py res_ln)
        # (an emulated rank -- parallel/tp_emulation.py -- whose group has a rank-local custom all-reduce
        # registered runs the same kernels: bench/bloom_tp_bench.py measures the deployment's launches)
        self._tp_ar = None
        if (tp and self._layer_kind == "seq"
                and os.environ.get("KCA_TP_FUSED_TAIL", "1") not in ("0", "false")):
            from ..parallel.custom_ar import lookup
            ars = {id(mm.group): lookup(mm.group) for mm in rows}
            if len(ars) == 1 and None not in ars.values():
                self._tp_ar = next(iter(ars.values()))
        self._fused_ok = (on_gpu and not self.multi_device and (not tp or tp_local or self._tp_ar is not None)
                          and os.environ.get("KCA_DECODE_FUSED", "1") not in ("0", "false")
                          and cfg.hidden <= 16384
                          and (self._layer_kind != "neox"
                               or all(x.eps == blk.ln_1.eps for x, blk in zip(ln2, model.h)))
                          and (self._layer_kind == "seq"
                               or (self.H == self.Hkv and self.D % 8 == 0 and 64 < self.D <= 256)))
        self._fz: dict = {}
        self.step_launches: dict = {}
        self._outbufs: dict = {}
        self._chain_src = None
        # the fused step head gathers the token embedding itself (no learned positions / scale / LN on
        # the embedding) and resolves chained tokens on the device: KCA_DECODE_EMBED_HEAD=0 keeps the
        # torch embedding + cast + LN launches
        # (BLOOM's embedding LayerNorm: the gather kernel normalises with it, one ln_rows launch follows)
        self._embed_head = (self._fused_ok and getattr(model, "wpe", None) is None and cfg.embed_scale == 1.0
                            and os.environ.get("KCA_DECODE_EMBED_HEAD", "1") not in ("0", "false"))
        # batch 2..64: the matrix-core decode layer (ops/skinny_mm.py): every projection one weight-streaming
        # MFMA launch with its epilogue fused -- LayerNorm applied to the activation on load from the row
        # statistics the previous residual projection published, bias + GELU, bias + residual -- so the
        # layer loop has no LayerNorm, bias or hipBLASLt launch (parallel residual: [QKV | fc_in] one launch,
        # out-proj + fc_out one K-concatenated launch). KCA_DECODE_FUSED_BATCHED=0: per-projection path.
        d_model = cfg.hidden
        self.batched_steps = 0
        self._packs = {}  # packed weight twins of the matrix-core layer (_packed_w)
        self.fused_steps = 0  # batch-1 fused-layer steps built (eager runs and graph captures)
        # (real TP: sequential layers only -- each row-parallel projection closed by the custom all-reduce's
        # residual + row-statistics tail, parallel/custom_ar.py res_stats)
        # fp16 (the precision FasterTransformer / DS-Inference serve, BASELINE config 4) runs the same two
        # layers: every decode kernel (GEMVs, fused tails, attention, LayerNorm rows, MFMA layer, all-reduce
        # tails, sampler) has an fp16 instantiation (the *_f16 entry points)
        self._batched_ok = (self._fused_ok and self.dtype in (torch.bfloat16, torch.float16)
                            and d_model % 64 == 0 and d_model <= 16384
                            and os.environ.get("KCA_DECODE_FUSED_BATCHED", "1") not in ("0", "false"))
        # largest batch bucket the matrix-core layer takes, per layer kind, from same-box A/Bs against the
        # per-projection path (hipBLASLt + the fused LN / GELU / all-reduce launches,
        # profiles/decode_suite_r6_batched_vs_unfused.jsonl): GPT-J 3.49 vs 3.88 ms at B=16 but 4.63 vs
        # 4.27 at 32 (the per-projection step overlaps the MLP GEMMs with the attention on a side stream);
        # BLOOM TP=8 rank 11.46 vs 12.58 at 16, 14.25 vs 13.50 at 32 (hipBLASLt streams the 14336-wide
        # shapes faster from M = 32); NeoX wins at every batch (12.84 vs 15.86 at 32, 25.9 vs 28.3 at 64)
        # fp16 takes the same caps since the per-projection path's LayerNorm / GELU run their fp16
        # instantiations (ln_rows, kca_gelu_fwd_f16) instead of eager kernels: B=32 GPT-J 4.40 vs 4.65 ms,
        # BLOOM rank 13.38 vs 14.84 per-projection vs matrix-core layer (profiles/decode_fp16_cap_ab_r6.jsonl)
        self._batched_max_b = int(os.environ.get("KCA_DECODE_BATCHED_MAX_B", "0")) or \
            {"gptj": 16, "seq": 16}.get(self._layer_kind, 64)

    # ------------------------------------------------------------- prefill
    @torch.no_grad()
    def prefill(self, ids: torch.Tensor, slots: list[int], lens: list[int] | None = None,
                start: list[int] | None = None) -> torch.Tensor:
        """ids [n, T] prompts, right-padded to T when ``lens`` (their true
        lengths) is given -> last-real-position logits [n, V]. Writes K/V of
        positions [0, lens[i]) into each slot and marks the prompt as seen.
        Padding needs no mask: with causal attention a real query row never
        sees a key to its right, so ragged prompts batch into one pass.

        ``start`` (chunked prefill): row i continues slot i's sequence at
        position start[i] -- its K/V land at [start, start + lens[i]) and its
        queries attend to the cached prefix plus the chunk."""
        m, cfg = self.model, self.cfg
        ids = ids.to(self.device)
        n, T = ids.shape
        lens = [T] * n if lens is None else [int(x) for x in lens]
        start = [0] * n if start is None else [int(x) for x in start]
        assert len(lens) == n and len(start) == n and all(0 < L <= T for L in lens)
        assert all(p0 + L <= self.max_len for p0, L in zip(start, lens))
        ragged = any(L != T for L in lens)
        cont = any(start)
        for s_, L, p0 in zip(slots, lens, start):
            if p0 == 0:
                self.cache.release(s_)  # a reused slot starts empty
            self.cache.reserve(s_, p0 + L)
        self.cache.sync()
        plan = self.cache.plan_write(slots, lens, T, start)
        sl = torch.tensor(slots, device=self.device, dtype=torch.long)
        fresh = [i for i, p0 in enumerate(start) if p0 == 0]
        if len(fresh) == n:
            self.seen[sl] = 0
        elif fresh:
            self.seen[sl[fresh]] = 0
        if ragged:
            valid = torch.arange(T, device=self.device)[None] < torch.tensor(lens, device=self.device)[:, None]
            self.seen[sl[:, None].expand(n, T)[valid], ids[valid]] = 1
        else:
            self.seen[sl[:, None].expand(n, T), ids] = 1
        pos_ids = None
        if cont:
            pos_ids = (torch.tensor(start, device=self.device)[:, None]
                       + torch.arange(T, device=self.device)[None]).clamp_(max=self.max_len - 1)
        h = m.embed(ids, pos_ids if cont else None)
        pending = ()
        for li, blk in enumerate(m.h):
            if self.multi_device and h.device != self.layer_devs[li]:
                h, pending = self._hop(self.layer_devs[li], h, pending)
            x, h = blk.ln_1(h, residual=pending) if pending else (blk.ln_1(h), h)
            at = blk.attn
            qkv = at.qkv(x).view(n, T, 3, self.H, self.D)
            q, k, v = qkv[:, :, 0], qkv[:, :, 1], qkv[:, :, 2]
            if self.rot > 0:
                ops.apply_rotary_(q, k, self.rot, T, cfg.rotary_interleaved, cfg.rotary_base,
                                  pos_ids=pos_ids, max_pos=self.max_len)
            self.cache.write(li, k, v, slots, lens, plan, start)
            if cont:
                o = self._continued_attention(li, q, slots, lens, start, at)
            else:  # (GPT-Neo local layers: banded, the kernels skip the tiles left of the band)
                o = ops.flash_attention(q, k, v, causal=True, scale=at.scale, alibi=at.alibi, window=at.window)
            a = at.out(o.reshape(n, T, -1))
            if cfg.parallel_residual:
                x2 = x if blk.ln_2 is None else blk.ln_2(h)
                pending = (a, blk.mlp(x2))
            else:
                x2, h = blk.ln_2(h, residual=(a,))
                pending = (blk.mlp(x2),)
        if self.multi_device and h.device != self.head_dev:
            h, pending = self._hop(self.head_dev, h, pending)
        if ragged:
            rows = torch.arange(n, device=h.device)
            last = torch.tensor(lens, device=h.device) - 1
            pick = lambda t: t[rows, last][:, None]  # noqa: E731
        else:
            pick = lambda t: t[:, -1:]  # noqa: E731
        y, _ = m.ln_f(pick(h), residual=tuple(pick(p_) for p_ in pending))
        return m.logits_from_hidden(y)[:, -1].to(self.device)

    def _continued_attention(self, li, q, slots, lens, start, at):
        """Chunk queries [start, start + L) of each row against the slot's cached
        keys [0, start + L) (just written): bottom-right-aligned causal mask,
        so query j of the chunk sees keys <= start + j."""
        n, T = q.shape[0], q.shape[1]
        o = torch.zeros_like(q)
        kc, vc, tbl = self.cache.k[li], self.cache.v[li], self.cache.table_on(self.layer_devs[li])
        for i, (s_, L, p0) in enumerate(zip(slots, lens, start)):
            kv = p0 + L
            lo = max(0, kv - L - at.window + 1) if at.window else 0  # oldest key any chunk query can see
            kw = dops.gather_kv(kc, s_, kv, tbl)[:, lo:].transpose(0, 1)[None]
            vw = dops.gather_kv(vc, s_, kv, tbl)[:, lo:].transpose(0, 1)[None]
            o[i:i + 1, :L] = ops.flash_attention(q[i:i + 1, :L], kw, vw, causal=True, scale=at.scale,
                                                 alibi=at.alibi, window=at.window)
        return o

    @staticmethod
    def _hop(dev, h, pending):
        """Move the residual stream to the next layer-split device."""
        return h.to(dev), tuple(p_.to(dev) for p_ in pending)

    # -------------------------------------------------------------- decode
    def _fused_bufs(self):
        """Static buffers of the fused batch-1 layer (allocated outside any graph capture)."""
        fz = self._fz.get("b1")
        if fz is None:
            d, f = self.cfg.hidden, self.model.h[0].mlp.fc_in.weight.shape[0]
            z = dict(device=self.device, dtype=self.dtype)
            biases = []
            for blk in self.model.h:
                bo, bf = blk.attn.out.bias, blk.mlp.fc_out.bias
                biases.append(bf if bo is None else (bo if bf is None else (bo.float() + bf.float()).to(self.dtype)))
            fz = self._fz["b1"] = {
                "g": torch.empty(1, f, **z), "h": torch.empty(1, d, **z), "xn": torch.empty(1, d, **z),
                "xn2": torch.empty(1, d, **z), "ypart": torch.empty(d, device=self.device, dtype=torch.float32),
                "cnt": torch.zeros(32 * 65, device=self.device, dtype=torch.int32), "bias": biases}
        return fz

    def _desc_args(self, cos, sin, tbl):
        """(cos, sin, block table, by_row) for the decode attention: the step descriptors' rows where
        this step has them (see _STEP_DESC), else the position tables and the device block table."""
        by_row = 0
        if self._step_desc is not None:
            rc, rs, pages = self._step_desc
            if rc is not None and cos is not None:
                cos, sin, by_row = rc, rs, 1
            if pages is not None and tbl is not None:
                tbl, by_row = pages, by_row | 2
        return cos, sin, tbl, by_row

    def _layers_decode_fused(self, tokens, pos, slots, kv_lens, max_kv, ws, obuf):
        """Batch-1 decode step, one queue, the residual + next LayerNorm in each layer's last projection
        (see _fused_ok for the three layer kinds). Returns None (nothing launched) when the fused kernels
        do not cover the shape."""
        m, cfg = self.model, self.cfg
        fz = self._fused_bufs()
        kind = self._layer_kind
        blk0 = m.h[0]
        if self._embed_head:  # token gather (+ chained token) + LayerNorm: one kernel
            chain, prev = self._chain_src if self._chain_src is not None else (None, None)
            if m.emb_ln is not None:  # BLOOM: the residual stream starts at LN_emb(wte[id])
                h, _ = embed_ln_rows(m.wte.weight, tokens, m.emb_ln.weight, m.emb_ln.bias, m.emb_ln.eps,
                                     chain=chain, prev=prev)
                xn, _ = ln_rows(h, blk0.ln_1.weight, blk0.ln_1.bias, blk0.ln_1.eps)
            else:
                xn, h = embed_ln_rows(m.wte.weight, tokens, blk0.ln_1.weight, blk0.ln_1.bias, blk0.ln_1.eps,
                                      chain=chain, prev=prev)
        else:
            h0 = m.embed(tokens, pos.long())
            xn, h = ln_rows(h0, blk0.ln_1.weight, blk0.ln_1.bias, blk0.ln_1.eps)
        xn2 = ln_rows(h, blk0.ln_2.weight, blk0.ln_2.bias, blk0.ln_2.eps)[0] if kind == "neox" else None
        hb, xb, x2b, g = fz["h"], fz["xn"], fz["xn2"], fz["g"]
        tbl = self.cache.table_on(self.device)
        cos, sin, tbl, by_row = self._desc_args(self.cos, self.sin, tbl)
        for li, blk in enumerate(m.h):
            at, mlp = blk.attn, blk.mlp
            act = 1 if mlp.approx in ("tanh", True) else 2
            kc, vc = self.cache.k[li], self.cache.v[li]
            nxt = m.h[li + 1] if li + 1 < len(m.h) else None
            nln = nxt.ln_1 if nxt is not None else m.ln_f
            qkv = skinny_linear(xn, at.qkv.weight, at.qkv.bias)
            if kind == "seq" and self._tp_ar is not None:
                # TP rank: partial projections, each closed by all-reduce + bias + residual + LayerNorm
                ar = self._tp_ar
                o = dops.decode_prep_attention(qkv, self.H, self.Hkv, self.D, self.rot, cfg.rotary_interleaved,
                                               cos, sin, pos, slots, kc, vc, kv_lens, max_kv, at.scale, at.alibi,
                                               out=obuf, ws=ws, block_table=tbl, window=at.window, by_row=by_row)
                ar.res_ln(skinny_linear(o, at.out.weight), at.out.bias, h, hb, blk.ln_2.weight, blk.ln_2.bias,
                          blk.ln_2.eps, x2b)
                f = skinny_linear(x2b, mlp.fc_in.weight, mlp.fc_in.bias, act, out=g)
                ar.res_ln(skinny_linear(f, mlp.fc_out.weight), mlp.fc_out.bias, hb, hb, nln.weight, nln.bias,
                          nln.eps, xb)
                h, xn = hb, xb
                continue
            if kind == "seq":
                # attention, out-projection + residual + ln_2, fc_in (+ GELU), fc_out + residual + next ln_1
                # (a fused attention + out-projection launch and tail launches chained with the next
                # projection measured slower: profiles/decode_launch_structure_ab_r5.txt)
                o = dops.decode_prep_attention(qkv, self.H, self.Hkv, self.D, self.rot, cfg.rotary_interleaved,
                                               cos, sin, pos, slots, kc, vc, kv_lens, max_kv, at.scale, at.alibi,
                                               out=obuf, ws=ws, block_table=tbl, window=at.window, by_row=by_row)
                dops.gemv_dual_ln(o, at.out.weight, None, None, at.out.bias, h, blk.ln_2.weight, blk.ln_2.bias,
                                  blk.ln_2.eps, fz["ypart"], fz["cnt"], hb, x2b)
                f = skinny_linear(x2b, mlp.fc_in.weight, mlp.fc_in.bias, act, out=g)
                dops.gemv_dual_ln(f, mlp.fc_out.weight, None, None, mlp.fc_out.bias, hb, nln.weight, nln.bias,
                                  nln.eps, fz["ypart"], fz["cnt"], hb, xb)
                h, xn = hb, xb
                continue
            # parallel residual: attention + fc_in (of ln_2's output for NeoX) in one launch
            if not dops.decode_prep_attention_gemv(
                    qkv, self.H, self.Hkv, self.D, self.rot, cfg.rotary_interleaved, cos, sin, pos, slots, kc, vc,
                    kv_lens, max_kv, at.scale, at.alibi, obuf, ws, tbl, at.window,
                    xn2 if kind == "neox" else xn, mlp.fc_in.weight, mlp.fc_in.bias, g, act, by_row):
                if li == 0:
                    return None
                raise RuntimeError("fused decode layer: shape support changed between layers")
            two = kind == "neox" and nxt is not None
            dops.gemv_dual_ln(obuf, at.out.weight, g, mlp.fc_out.weight, fz["bias"][li], h, nln.weight, nln.bias,
                              nln.eps, fz["ypart"], fz["cnt"], hb, xb,
                              *((nxt.ln_2.weight, nxt.ln_2.bias, x2b) if two else ()))
            h, xn, xn2 = hb, xb, (x2b if two else None)
        if m.lm_head is None:
            return skinny_linear(xn, m.wte.weight)
        return self._lin(m.lm_head, xn)

    def _batched_bufs(self, B: int):
        """Static buffers of the batched matrix-core layer for a batch bucket (outside graph capture)."""
        key = ("mm", B)
        fz = self._fz.get(key)
        if fz is None:
            m = self.model
            d = self.cfg.hidden
            at0, mlp0 = m.h[0].attn, m.h[0].mlp
            z = dict(device=self.device, dtype=self.dtype)
            biases = []
            for blk in m.h:
                bo, bf = blk.attn.out.bias, blk.mlp.fc_out.bias
                biases.append(bf if bo is None else (bo if bf is None else (bo.float() + bf.float()).to(self.dtype)))
            fz = self._fz[key] = {
                "h": torch.empty(B, d, **z), "xn": torch.empty(B, d, **z), "xn2": torch.empty(B, d, **z),
                "qkv": torch.empty(B, at0.qkv.weight.shape[0], **z), "g": torch.empty(B, mlp0.fc_in.weight.shape[0], **z),
                "y": torch.empty(B, d, **z),  # a TP rank's partial projection before the all-reduce
                "st": smm.RowStatsBuf(B, d, self.device), "bias": biases}
        return fz

    def _head_weight(self):
        from ..parallel.tensor_parallel import ParallelLMHead
        m = self.model
        if m.lm_head is None:
            return m.wte.weight, None, None
        if isinstance(m.lm_head, ParallelLMHead):
            return m.lm_head.local_weight(), m.lm_head.bias, m.lm_head.group
        return m.lm_head.weight, m.lm_head.bias, None

    def _layers_decode_batched(self, tokens, pos, slots, kv_lens, max_kv, ws, obuf):
        """Decode step at batch 2..64 on the matrix cores (see _batched_ok). Per layer kind:
          seq  : QKV(LN1 on load) -> attention -> out + b + h (stats) -> fc_in(LN2 on load, GELU) -> fc_out + b + h
          gptj : [QKV | fc_in+GELU](LN1 on load) -> attention -> o.Wo + g.Wf + b + h (stats)
          neox : as gptj, fc_in normalising with ln_2's gamma / beta (same statistics)
        Layer 0 reads the step head's normalised rows; the LM head normalises with ln_f on load."""
        m, cfg = self.model, self.cfg
        B = tokens.shape[0]
        fz = self._batched_bufs(B)
        self.batched_steps += 1  # (counted when a step is built: eager runs and graph captures)
        kind = self._layer_kind
        blk0 = m.h[0]
        hb, st, qkv, g = fz["h"], fz["st"], fz["qkv"], fz["g"]
        dt = self.dtype
        # step head: token rows (+ BLOOM's embedding LayerNorm) and ln_1 (+ ln_2 for NeoX) of layer 0
        if self._embed_head:  # (resolves a chained token of the previous step on the device, as at B = 1)
            chain, prev = self._chain_src if self._chain_src is not None else (None, None)
            if m.emb_ln is not None:
                h, _ = embed_ln_rows(m.wte.weight, tokens, m.emb_ln.weight, m.emb_ln.bias, m.emb_ln.eps,
                                     chain=chain, prev=prev)
                xn, h = ln_rows(h, blk0.ln_1.weight, blk0.ln_1.bias, blk0.ln_1.eps)
            else:
                xn, h = embed_ln_rows(m.wte.weight, tokens, blk0.ln_1.weight, blk0.ln_1.bias, blk0.ln_1.eps,
                                      chain=chain, prev=prev)
        else:
            xn, h = ln_rows(m.embed(tokens, pos.long()), blk0.ln_1.weight, blk0.ln_1.bias, blk0.ln_1.eps)
        xn2 = ln_rows(h, blk0.ln_2.weight, blk0.ln_2.bias, blk0.ln_2.eps)[0] if kind == "neox" else None
        hb.copy_(h)
        tbl = self.cache.table_on(self.device)
        cos, sin, tbl, by_row = self._desc_args(self.cos, self.sin, tbl)
        pk = self._packed_w

        def part(x, w, ln=None):  # one K-part, streaming the weight's packed twin
            return smm.part(x, w, ln, packed=pk(w))

        for li, blk in enumerate(m.h):
            at, mlp = blk.attn, blk.mlp
            act = 1 if mlp.approx in ("tanh", True) else 2
            nxt = m.h[li + 1] if li + 1 < len(m.h) else None
            nln = nxt.ln_1 if nxt is not None else m.ln_f
            first = li == 0
            ln1 = None if first else (st, blk.ln_1.weight, blk.ln_1.bias)
            x1 = xn if first else hb
            kc, vc = self.cache.k[li], self.cache.v[li]
            if kind == "seq" and self._tp_ar is not None:
                # TP rank: partial projections, each closed by all-reduce + bias + residual + row statistics
                ar, y = self._tp_ar, fz["y"]
                smm.launch([smm.job([part(x1, at.qkv.weight, ln1)], qkv.shape[1], qkv, at.qkv.bias)], B, dt)
                o = dops.decode_prep_attention(qkv, self.H, self.Hkv, self.D, self.rot, cfg.rotary_interleaved,
                                               cos, sin, pos, slots, kc, vc, kv_lens, max_kv, at.scale, at.alibi,
                                               out=obuf, ws=ws, block_table=tbl, window=at.window, by_row=by_row)
                smm.mm(o, at.out.weight, out=y, packed=pk(at.out.weight))
                ar.res_stats(y, at.out.bias, hb, hb, st, blk.ln_2.eps)
                smm.launch([smm.job([part(hb, mlp.fc_in.weight, (st, blk.ln_2.weight, blk.ln_2.bias))],
                                    g.shape[1], g, mlp.fc_in.bias, act)], B, dt)
                smm.mm(g, mlp.fc_out.weight, out=y, packed=pk(mlp.fc_out.weight))
                ar.res_stats(y, mlp.fc_out.bias, hb, hb, st, nln.eps)
                continue
            if kind == "seq":
                smm.launch([smm.job([part(x1, at.qkv.weight, ln1)], qkv.shape[1], qkv, at.qkv.bias)], B, dt)
                o = dops.decode_prep_attention(qkv, self.H, self.Hkv, self.D, self.rot, cfg.rotary_interleaved,
                                               cos, sin, pos, slots, kc, vc, kv_lens, max_kv, at.scale, at.alibi,
                                               out=obuf, ws=ws, block_table=tbl, window=at.window, by_row=by_row)
                smm.launch([smm.job([part(o, at.out.weight)], hb.shape[1], hb, at.out.bias, res=hb, stats=st,
                                    eps=blk.ln_2.eps)], B, dt)
                smm.launch([smm.job([part(hb, mlp.fc_in.weight, (st, blk.ln_2.weight, blk.ln_2.bias))],
                                    g.shape[1], g, mlp.fc_in.bias, act)], B, dt)
                smm.launch([smm.job([part(g, mlp.fc_out.weight)], hb.shape[1], hb, mlp.fc_out.bias, res=hb,
                                    stats=st, eps=nln.eps)], B, dt)
                continue
            # parallel residual: [QKV | fc_in] of the same residual rows, one launch
            if kind == "neox":
                ln2 = (st, blk.ln_2.weight, blk.ln_2.bias) if not first else None
                x2 = xn2 if first else hb
            else:
                ln2, x2 = ln1, x1
            smm.launch([smm.job([part(x1, at.qkv.weight, ln1)], qkv.shape[1], qkv, at.qkv.bias),
                        smm.job([part(x2, mlp.fc_in.weight, ln2)], g.shape[1], g, mlp.fc_in.bias, act)], B, dt)
            o = dops.decode_prep_attention(qkv, self.H, self.Hkv, self.D, self.rot, cfg.rotary_interleaved,
                                           cos, sin, pos, slots, kc, vc, kv_lens, max_kv, at.scale, at.alibi,
                                           out=obuf, ws=ws, block_table=tbl, window=at.window, by_row=by_row)
            smm.launch([smm.job([part(o, at.out.weight), part(g, mlp.fc_out.weight)], hb.shape[1], hb,
                                fz["bias"][li], res=hb, stats=st, eps=nln.eps)], B, dt)
        w, b, grp = self._head_weight()
        V = w.shape[0]
        if V % 4 == 0:
            logits = smm.mm(hb, w, b, ln=(st, m.ln_f.weight, m.ln_f.bias), packed=pk(w))
        else:  # (GPT-2's 50257 rows: the head takes the normalised rows through the plain path)
            y = smm.ln_on_load_reference(hb, st.merged(hb.shape[0]), m.ln_f.weight, m.ln_f.bias)
            logits = skinny_linear(y, w, b)
        if grp is not None:
            from ..parallel.tensor_parallel import gather_last_dim
            logits = gather_last_dim(logits, grp)
        return logits

    def _packed_w(self, w):
        """The packed stream twin of a weight the matrix-core layer reads (``skinny_mm.pack_weight``):
        built once, on the first (eager) step that uses it -- the graph-capture warm-up -- and kept for the
        runner's life (KCA_MM_PACK=0: none, the row-major weight streams). Keyed by storage address,
        shape and version (an in-place weight update re-packs)."""
        if not smm.PACK:
            return None
        key = (w.data_ptr(), tuple(w.shape), w._version)
        p = self._packs.get(key)
        if p is None and not torch.cuda.is_current_stream_capturing():
            p = self._packs[key] = smm.pack_weight(w.detach())
        return p

    def _layers_decode(self, tokens, pos, slots, kv_lens, max_kv, ws, obuf):
        m, cfg = self.model, self.cfg
        if self._fused_ok and tokens.shape[0] == 1 and obuf is not None:
            y = self._layers_decode_fused(tokens, pos, slots, kv_lens, max_kv, ws, obuf)
            if y is not None:
                self.fused_steps += 1
                return y
        if (self._batched_ok and 2 <= tokens.shape[0] <= min(smm.MAX_M, self._batched_max_b) and obuf is not None
                and (self._chain_src is None or self._embed_head)):
            return self._layers_decode_batched(tokens, pos, slots, kv_lens, max_kv, ws, obuf)
        if self._chain_src is not None and obuf is not None:  # chained rows not resolved by a fused head
            chain, prev = self._chain_src
            tokens = torch.where(chain[:tokens.shape[0]] >= 0, prev[chain[:tokens.shape[0]].clamp(min=0).long()],
                                 tokens)
        h = m.embed(tokens, pos.long())
        pending = ()
        per_dev = {self.device: (pos, slots, kv_lens, ws, obuf)}
        for li, blk in enumerate(m.h):
            # every LayerNorm (+ pending residual adds) runs as the prologue of the GEMM that consumes it
            at = blk.attn
            dev = self.layer_devs[li]
            if self.multi_device:
                if h.device != dev:
                    h, pending = self._hop(dev, h, pending)
                if dev not in per_dev:
                    per_dev[dev] = (pos.to(dev), slots.to(dev), kv_lens.to(dev), None, None)
                pos, slots, kv_lens, ws, obuf = per_dev[dev]
            shared = cfg.parallel_residual and blk.ln_2 is None  # GPT-J: one LN feeds qkv and fc_in
            # (forking before the QKV GEMV was measured slower at B=1, 3.09 vs 2.99 ms on one box: the
            # QKV GEMV then shares HBM with the MLP GEMVs and the attention chain starts later)
            if shared:
                qkv, h, xn = self._ln_lin(blk.ln_1, h, pending, at.qkv, want_xn=True)
            else:
                qkv, h = self._ln_lin(blk.ln_1, h, pending, at.qkv)
            mlp = blk.mlp
            act = 1 if mlp.approx in ("tanh", True) else 2
            side_out = None
            if self._par_mlp:  # fork: MLP branch on the side stream
                cur = torch.cuda.current_stream()
                self._side.wait_stream(cur)
                with torch.cuda.stream(self._side):
                    if shared:
                        xm = xn
                    else:
                        xm, _ = self._ln_lin(blk.ln_2, h, (), mlp.fc_in, act)  # NeoX: ln_2 + fc_in fused
                    side_out = self._lin(mlp.fc_out, self._lin(mlp.fc_in, xm, act) if shared else xm)
                if not torch.cuda.is_current_stream_capturing():  # eager: keep cross-stream buffers alive
                    xm.record_stream(self._side)
                    h.record_stream(self._side)
            kc, vc, tbl = self.cache.k[li], self.cache.v[li], self.cache.table_on(dev)
            cos, sin = self._rope[dev]
            by_row = 0
            if obuf is not None and not self.multi_device:  # a graph-bucket step: its descriptors
                cos, sin, tbl, by_row = self._desc_args(cos, sin, tbl)
            # RoPE + cache append + split-K attention (one launch on the GPU; GPT-Neo local layers read
            # only the last `window` positions)
            o = dops.decode_prep_attention(qkv, self.H, self.Hkv, self.D, self.rot, cfg.rotary_interleaved,
                                           cos, sin, pos, slots, kc, vc, kv_lens, max_kv, at.scale, at.alibi,
                                           out=obuf, ws=ws, block_table=tbl, window=at.window, by_row=by_row)
            a = self._lin(at.out, o)
            if side_out is not None:  # join
                cur.wait_stream(self._side)
                if not torch.cuda.is_current_stream_capturing():
                    side_out.record_stream(cur)
                pending = (a, side_out)
            elif shared:
                pending = (a, self._lin(mlp.fc_out, self._lin(mlp.fc_in, xn, act)))
            elif cfg.parallel_residual:
                f, _ = self._ln_lin(blk.ln_2, h, (), mlp.fc_in, act)
                pending = (a, self._lin(mlp.fc_out, f))
            else:
                f, h = self._ln_lin(blk.ln_2, h, (a,), mlp.fc_in, act)
                pending = (self._lin(mlp.fc_out, f),)
        if self.multi_device and h.device != self.head_dev:
            h, pending = self._hop(self.head_dev, h, pending)
        if m.lm_head is None:
            y = self._ln_lin(m.ln_f, h, pending, None, weight=m.wte.weight)[0]
        else:
            y = self._ln_lin(m.ln_f, h, pending, m.lm_head)[0]
        return y.to(self.device) if self.multi_device else y

    def _ln_lin(self, ln, h, res, mod, act: int = 0, weight=None, want_xn: bool = False):
        """LayerNorm(h + sum(res)) -> column-parallel / LM-head linear, fused (decode)."""
        from ..parallel.tensor_parallel import ParallelLMHead, RowParallelLinear, gather_last_dim
        assert not isinstance(mod, RowParallelLinear)
        if isinstance(mod, ParallelLMHead):
            y, h = ln_skinny_linear(h, ln.weight, ln.bias, ln.eps, mod.local_weight(), mod.bias, res, act)
            return gather_last_dim(y, mod.group), h
        return ln_skinny_linear(h, ln.weight, ln.bias, ln.eps, mod.weight if weight is None else weight,
                                None if mod is None else mod.bias, res, act, want_xn=want_xn)

    # decode linears: skinny GEMM (W streamed once, bias/GELU fused) for <= 16 rows
    def _lin(self, mod, x, act: int = 0):
        from ..parallel.tensor_parallel import ParallelLMHead, RowParallelLinear, gather_last_dim, reduce_from_tp
        if isinstance(mod, RowParallelLinear):
            y = reduce_from_tp(skinny_linear(x, mod.weight, None), mod.group)
            return y + mod.bias if mod.bias is not None else y
        if isinstance(mod, ParallelLMHead):
            return gather_last_dim(skinny_linear(x, mod.local_weight(), mod.bias), mod.group)
        return skinny_linear(x, mod.weight, mod.bias, act)

    def _static_for(self, Bb: int, Kb: int):
        key = (Bb, Kb)
        st = self._static.get(key)
        if st is not None:
            return st
        NB = self.max_bans
        pk = _Packed({"tokens": (torch.int64, Bb), "seeds": (torch.int64, Bb), "pos": (torch.int32, Bb),
                      "slots": (torch.int32, Bb), "kv_lens": (torch.int32, Bb), "top_k": (torch.int32, Bb),
                      "temperature": (torch.float32, Bb), "top_p": (torch.float32, Bb),
                      "rep": (torch.float32, Bb), "bans": (torch.int32, Bb * NB),
                      "chain": (torch.int32, Bb), **self._desc_fields(Bb)}, self.device)
        ws_n = dops.decode_ws_floats(Bb, self.H, self.Hkv, self.D, Kb)
        ob = self._outbuf(Bb)
        st = {
            "pk": pk,
            "ws": torch.zeros(max(ws_n, 1), device=self.device, dtype=torch.float32),  # zeroed: fan-in counters
            "obuf": torch.empty(Bb, self.H * self.D, device=self.device, dtype=self.dtype),
            "sws": torch.empty(Bb * self.V, device=self.device, dtype=torch.float32),
            **ob,
        }
        self._static[key] = st
        return st

    def _desc_on(self, Bb: int) -> bool:
        return (_STEP_DESC and (Bb == 1 or _STEP_DESC_BATCHED) and self.device.type == "cuda"
                and not self.multi_device and (self.rot > 0 or self.cache.paged))

    def _desc_fields(self, Bb: int) -> dict:
        """Per-step descriptor arrays (see _STEP_DESC): row i's RoPE angles and page-table row."""
        if not self._desc_on(Bb):
            return {}
        f = {}
        if self.rot > 0:
            f["rcos"] = (torch.float32, Bb * (self.rot // 2))
            f["rsin"] = (torch.float32, Bb * (self.rot // 2))
        if self.cache.paged:
            f["pages"] = (torch.int32, Bb * self.cache.blocks)
        return f

    def _fill_desc(self, a, Bb: int, pos, slots):
        """Host side of the step descriptors: row i's RoPE angles at its position and its page row."""
        if "rcos" in a:
            half = self.rot // 2
            ch, sh = self._rope_h
            a["rcos"].reshape(Bb, half)[:] = ch[pos[:Bb]]
            a["rsin"].reshape(Bb, half)[:] = sh[pos[:Bb]]
        if "pages" in a:
            a["pages"].reshape(Bb, self.cache.blocks)[:] = self.cache.table_h.numpy()[slots[:Bb]]

    def _desc_views(self, pk, Bb: int):
        """(cos rows, sin rows, page rows) device views of the step descriptors (None where absent)."""
        f = pk.fields
        return (pk.d("rcos") if "rcos" in f else None, pk.d("rsin") if "rsin" in f else None,
                pk.d("pages").view(Bb, self.cache.blocks) if "pages" in f else None)

    def _outbuf(self, Bb: int):
        """Sampled ids (int64) and log-probs (fp32) of a batch bucket in ONE device buffer shared by its
        kv-length buckets -- one D2H copy per step, and a chained token (decode_async) is read by the
        next step's embedding kernel from a fixed address whatever kv bucket that step lands in --
        with two pinned landing buffers (one per host pk buffer)."""
        ob = self._outbufs.get(Bb)
        if ob is None:
            pin = self.device.type == "cuda"
            dev = torch.empty(3 * Bb, device=self.device, dtype=torch.int32)
            hs = [torch.empty(3 * Bb, dtype=torch.int32, pin_memory=pin) for _ in range(2)]
            # "flip": the landing buffer of the latest launch, counted per BATCH bucket (every kv bucket of
            # this Bb copies into these two buffers, so consecutive launches must alternate here even when
            # they land in different kv buckets -- a per-(Bb, Kb) counter could hand two in-flight steps
            # the same buffer)
            ob = {"out": dev, "ids": dev[:2 * Bb].view(torch.int64), "lps": dev[2 * Bb:].view(torch.float32),
                  "flip": [0], "out_h": hs, "ids_h": [h[:2 * Bb].view(torch.int64) for h in hs],
                  "lps_h": [h[2 * Bb:].view(torch.float32) for h in hs]}
            self._outbufs[Bb] = ob
        return ob

    def _step_body(self, st, Bb, Kb, mc=False):
        n0 = _lib.LAUNCHES[0]
        try:
            self._step_body_inner(st, Bb, Kb, mc)
        finally:
            # native launches one decode step issues (counted when the step is built: eager, or graph capture)
            self.step_launches[Bb] = _lib.LAUNCHES[0] - n0

    def _step_body_inner(self, st, Bb, Kb, mc=False):
        pk = st["pk"]
        # chained tokens resolved on the device by the fused B = 1 step head (_layers_decode_fused)
        self._chain_src = (pk.d("chain"), st["ids"]) if (Bb == 1 and self._embed_head) else None
        if "rcos" in pk.fields or "pages" in pk.fields:
            self._step_desc = self._desc_views(pk, Bb)
        try:
            logits = self._layers_decode(pk.d("tokens"), pk.d("pos"), pk.d("slots"), pk.d("kv_lens"), Kb,
                                         st["ws"], st["obuf"])
        finally:
            self._step_desc = None
        dops.sample_logits(logits, temperature=pk.d("temperature"), top_k=pk.d("top_k"), top_p=pk.d("top_p"),
                           rep_penalty=pk.d("rep"), seen=self.seen, slots=pk.d("slots"),
                           ban_ids=pk.d("bans").view(Bb, self.max_bans), seeds=pk.d("seeds"), step=0,
                           ws=st["sws"], out_ids=st["ids"], out_logprobs=st["lps"], mwg_complete=mc)

    # ----------------------------------------------------------- beam search
    @torch.no_grad()
    def decode_topk(self, tokens: list[int], positions: list[int], slots: list[int], k: int):
        """Eager decode step returning the top-k next-token log-probs per row
        (beam search; K30). -> (logprobs [n, k] fp32, ids [n, k] int64) on device."""
        dev = self.device
        for s_, p_ in zip(slots, positions):
            self.cache.reserve(s_, p_ + 1)
        self.cache.sync()
        tok = torch.tensor(tokens, device=dev, dtype=torch.long)
        pos = torch.tensor(positions, device=dev, dtype=torch.int32)
        sl = torch.tensor(slots, device=dev, dtype=torch.int32)
        kl = pos + 1
        max_kv = max(positions) + 1
        logits = self._layers_decode(tok, pos, sl, kl, max_kv, None, None)
        lp = torch.log_softmax(logits.float(), dim=-1)
        return lp.topk(k, dim=-1)

    @torch.no_grad()
    def copy_slots(self, dst: list[int], src: list[int], upto: int):
        """KV cache (and seen mask) of ``src`` slots -> ``dst`` slots, positions
        [0, upto) (paged: prefix pages shared, see ``KVCache.fork``)."""
        if not dst:
            return
        self.cache.fork(dst, src, upto)
        self.cache.sync()
        d = torch.tensor(dst, device=self.device, dtype=torch.long)
        s = torch.tensor(src, device=self.device, dtype=torch.long)
        self.seen[d] = self.seen[s]

    def release(self, slot: int):
        """A finished sequence's KV pages go back to the pool."""
        self.cache.release(slot)

    pipelined = True  # supports decode_async (the TP CollectiveRunner does not)

    @torch.no_grad()
    def decode(self, rows: list[dict]):
        """rows: [{token, pos, slot, temperature, top_k, top_p, rep, seed, bans}]
        -> (ids list[int], logprobs list[float]) of the next token per row."""
        return self.decode_async(rows).result()

    @torch.no_grad()
    def decode_async(self, rows: list[dict], prev: DecodeHandle | None = None) -> DecodeHandle:
        """Launch one decode step without waiting for it. A row whose
        ``token`` is None takes its input token from ``prev``'s output row
        ``src`` on the device (the previous step's sample, not yet seen by the
        host), so the engine can launch step t+1 before reading step t: the GPU
        never idles on the host's bookkeeping between steps."""
        n = len(rows)
        Bb = _next_pow2(n)
        max_kv = max(r["pos"] for r in rows) + 1
        Kb = min(_next_pow2(max_kv, 256), self.max_len)
        if self.device.type != "cuda":
            Bb = n  # GPU eager keeps the graph buckets so both paths run identical shapes
        st = self._static_for(Bb, Kb)
        pk = st["pk"]
        pk.flip()
        NB = self.max_bans
        for r in rows:
            self.cache.reserve(r["slot"], r["pos"] + 1)
        self.cache.sync()
        a = pk.np
        tok, sd, pos, sl, kl = a["tokens"], a["seeds"], a["pos"], a["slots"], a["kv_lens"]
        tk, te, tp, rp, bans = a["top_k"], a["temperature"], a["top_p"], a["rep"], a["bans"]
        bans.fill(-1)
        ch = a["chain"]
        ch.fill(-1)
        chain_dst, chain_src = [], []
        for i in range(Bb):
            if i < n:
                r = rows[i]
                t = r["token"]
                if t is None:
                    chain_dst.append(i)
                    chain_src.append(int(r["src"]))
                    t = 0
                tok[i], pos[i], sl[i], kl[i] = t, r["pos"], r["slot"], r["pos"] + 1
                te[i], tk[i], tp[i], rp[i] = r["temperature"], r["top_k"], r["top_p"], r["rep"]
                sd[i] = r["seed"]
                b = r.get("bans") or ()
                if len(b) > NB:
                    raise ValueError(f"{len(b)} banned ids > max_bans={NB}")
                for j, t in enumerate(b):
                    bans[i * NB + j] = t
            else:  # padding row -> scratch slot
                tok[i], pos[i], sl[i], kl[i] = 0, 0, self.cache.scratch, 1
                te[i], tk[i], tp[i], rp[i], sd[i] = 0.0, 0, 1.0, 1.0, 0
        if "rcos" in pk.fields or "pages" in pk.fields:
            self._fill_desc(a, Bb, pos, sl)
        # every row (padding rows are greedy) on the multi-workgroup sampler: no closing kernel; the
        # step graphs are keyed by it too
        mc = bool(((~(te[:Bb] > 0)) | ((tk[:Bb] >= 1) & (tk[:Bb] <= dops.MWG_KMAX))).all())
        gk = (Bb, Kb, mc)
        if chain_dst and prev is None:
            raise ValueError("rows chain their token from a previous launch, but prev is None")
        # chained tokens read on the device by the step's first kernel: the previous step wrote them into
        # this bucket's shared output buffer (same batch bucket); otherwise copied into `tokens` below
        # (not on a step that captures its graph: the capture's eager warm-up runs would read the chained
        # token from the output buffer their own first run already overwrote)
        fold = (bool(chain_dst) and Bb == 1 and self._embed_head
                and prev.ids_dev.data_ptr() == st["ids"].data_ptr()
                and (not self.use_graphs or gk in self._graphs))
        if fold:
            for d_, s_ in zip(chain_dst, chain_src):
                ch[d_] = s_
        pk.upload()
        if chain_dst and not fold:
            dst = pk.d("tokens")
            m = len(chain_dst)
            if chain_dst == chain_src == list(range(m)):  # the common case: same rows, same order
                dst[:m].copy_(prev.ids_dev[:m])
            else:
                di = torch.tensor(chain_dst, dtype=torch.long).to(self.device, non_blocking=True)
                si = torch.tensor(chain_src, dtype=torch.long).to(self.device, non_blocking=True)
                dst.index_copy_(0, di, prev.ids_dev.index_select(0, si))
        if self.use_graphs:
            g = self._graphs.get(gk)
            if g is None:
                g = self._capture(st, Bb, Kb, mc)
            g.replay()
        else:
            self._step_body(st, Bb, Kb, mc)
        fl = st["flip"]
        fl[0] ^= 1
        k = fl[0]
        ids_h, lps_h = st["ids_h"][k], st["lps_h"][k]
        if self.device.type == "cuda":
            st["out_h"][k].copy_(st["out"], non_blocking=True)  # ids + log-probs, one copy
            ev = torch.cuda.Event()
            ev.record()
        else:
            st["out_h"][k].copy_(st["out"])
            ev = None
        return DecodeHandle(ids_h, lps_h, n, ev, st["ids"])

    def _capture(self, st, Bb, Kb, mc=False):
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            for _ in range(2):  # warm up (allocator, hipBLASLt heuristics)
                self._step_body(st, Bb, Kb, mc)
        torch.cuda.current_stream().wait_stream(s)
        if self._pool is None:
            self._pool = torch.cuda.graph_pool_handle()
        g = torch.cuda.CUDAGraph()
        # thread-local capture: the RCCL process-group watchdog thread polls its work events while a
        # capture runs; under the default global mode that query fails ("operation not permitted when
        # stream is capturing") and the watchdog aborts the process
        with torch.cuda.graph(g, pool=self._pool, capture_error_mode="thread_local"):
            self._step_body(st, Bb, Kb, mc)
        self._graphs[(Bb, Kb, mc)] = g
        return g

    @torch.no_grad()
    def sample_first(self, logits: torch.Tensor, rows: list[dict]):
        """Sample from prefill logits [n, V] (row params as in ``decode``)."""
        n = logits.shape[0]
        dev = self.device
        NB = self.max_bans
        bans = torch.full((n, NB), -1, dtype=torch.int32)
        for i, r in enumerate(rows):
            for j, t in enumerate((r.get("bans") or ())[:NB]):
                bans[i, j] = t
        f = lambda k, dt: torch.tensor([r[k] for r in rows], dtype=dt, device=dev)  # noqa: E731
        ids, lps = dops.sample_logits(
            logits.contiguous(), temperature=f("temperature", torch.float32), top_k=f("top_k", torch.int32),
            top_p=f("top_p", torch.float32), rep_penalty=f("rep", torch.float32), seen=self.seen,
            slots=f("slot", torch.int32), ban_ids=bans.to(dev), seeds=f("seed", torch.int64), step=0,
            mwg_complete=dops.mwg_complete_rows([r["temperature"] for r in rows], [r["top_k"] for r in rows]))
        return ids.tolist(), lps.tolist()


def mix_seed(seed: int, step: int) -> int:
    """Per-(request, token) 64-bit Philox key as a signed int64."""
    x = (seed * 0x9E3779B97F4A7C15 + (step + 1) * 0xBF58476D1CE4E5B9) & ((1 << 64) - 1)
    x ^= x >> 31
    x = (x * 0x94D049BB133111EB) & ((1 << 64) - 1)
    x ^= x >> 29
    return x - (1 << 64) if x >= (1 << 63) else x


__all__ = ["KVCache", "KVCacheFull", "ModelRunner", "DecodeHandle", "mix_seed", "math"]
