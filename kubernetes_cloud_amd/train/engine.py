"""Training engine: flat parameters, fp32 gradient accumulation, bucketed RCCL
collectives overlapped with backward, ZeRO stages 0-3, fused AdamW.

This is the MI355X-native replacement for the DeepSpeed ZeRO engine the
reference drives through HF Trainer (finetuner-workflow/finetuner/
ds_config.json:27-42: stage 3, reduce_bucket_size 2e8, overlap_comm,
reduce_scatter, contiguous_gradients, offload_optimizer/offload_param cpu,
stage3_gather_16bit_weights_on_model_save; finetuner.py:910-927 stage
override), for torch DDP / Horovod in the kubeflow examples
(resnet50_pytorch.py:121-122, resnet50_horovod.py:136-140) and for GPT-NeoX's
ZeRO-1 under PP x TP (gpt-neox/04-finetune-workflow.yaml:236-244).

Layout (every stage): each trainable parameter has a slot in ONE flat,
64-element-aligned index space, ordered for backward; slots are grouped into
buckets whose size is a multiple of 64*W so that rank r owns the contiguous
piece ``[start + r*size/W, start + (r+1)*size/W)`` of every bucket. A rank's
optimizer shard is the concatenation of its pieces, so a bucket's
reduce-scatter lands straight in that shard and one ``kca_adamw`` launch
updates it (fp32 master, clip + 1/W folded into a device scalar, no host sync).

Stages (W > 1; with W == 1 every stage runs as 0):

* 0 -- full bf16 params, full fp32 grads; bucket all-reduce in the last
  micro-batch's backward (DDP);
* 1 -- optimizer state sharded: bucket reduce-scatter in the last micro-batch's
  backward, AdamW on the shard, bf16 all-gather back into the flat params;
* 2 -- gradients sharded too: there is NO full fp32 gradient buffer. Every
  micro-batch, a bucket's grads accumulate into a transient bucket-sized
  staging buffer that is reduce-scattered as soon as the bucket is complete
  and added into the rank's fp32 grad shard; at most a few staging buffers are
  alive at a time;
* 3 -- parameters sharded too: a rank persistently holds only its bf16 piece
  (what AdamW writes). Buckets are *units* (a transformer block, the root
  embeddings/head); a unit's params are all-gathered into a transient buffer
  by a forward pre-hook (with the next unit prefetched on RCCL's stream),
  released by the forward post-hook, re-gathered by a backward pre-hook (with
  the previous unit prefetched) and released once the unit's gradients were
  reduce-scattered. Linear layers switch to an autograd function that saves
  the Parameter itself rather than a transposed view (a saved view would pin
  the gathered buffer for the whole forward). ``gathered()`` materialises the
  full model (checkpoint save with gather-16-bit-on-save, sampling);
  ``offload_param`` keeps the bf16 shard in pinned host memory.

Model parallelism (``set_model_parallel``): the clip norm sums over the
model-parallel group, with TP-replicated params counted once; works on the
full gradient or on the ZeRO shard (ranges are mapped into shard coordinates),
so ZeRO-1 runs over the DP group under TP x PP.
"""
from __future__ import annotations

import contextlib
import dataclasses
import functools
import logging
import os

import torch
import torch.distributed as dist
import torch.nn as nn

from ..ops import _lib, grad_sink
from .optim import FlatAdamW, FlatAdamW8bit, HostOffloadAdamW

log = logging.getLogger("kca.engine")

ALIGN = 64
_NONE, _INFLIGHT, _READY = 0, 1, 2
# gradients of at most this many elements are accumulated in batches (kca_accum_grad_multi);
# KCA_MULTI_ACCUM=0 launches kca_accum_grad per parameter
_SMALL_GRAD = 1 << 18
_MULTI_ACCUM = __import__("os").environ.get("KCA_MULTI_ACCUM", "1") not in ("0", "false")
# tests: KCA_DEFER_CPU=1 runs the batching logic on CPU tensors of any float dtype (torch-op flush)
_DEFER_CPU = __import__("os").environ.get("KCA_DEFER_CPU", "0") == "1"
_FLUSH_TORCH = __import__("os").environ.get("KCA_FLUSH_TORCH", "0") == "1"  # diagnostic: torch-op flush on GPU
# large bf16 gradients of the first micro-batch are kept until the second one's arrive and both go
# into the fp32 buffer in one pass (kca_accum_grad_pair); KCA_PAIR_ACCUM=0 accumulates each at once
_PAIR_ACCUM = __import__("os").environ.get("KCA_PAIR_ACCUM", "1") not in ("0", "false")
# the stash holds micro-batch 0's bf16 gradients until micro-batch 1 (2 bytes per stashed parameter): capped
# so a large model keeps the rest on the one-pass path (GPT-J: 12 GB fits; a NeoX-20B ZeRO-1 run would
# otherwise stash ~40 GB) -- KCA_PAIR_ACCUM_MAX_GB
_PAIR_ACCUM_MAX_BYTES = int(float(__import__("os").environ.get("KCA_PAIR_ACCUM_MAX_GB", "16")) * (1 << 30))


@dataclasses.dataclass
class ParamSlot:
    name: str
    param: nn.Parameter
    offset: int
    numel: int
    decay: bool
    bucket: int
    shape: tuple = ()


@dataclasses.dataclass
class Bucket:
    start: int
    size: int
    slots: list
    shard_off: int = 0  # offset of this rank's piece inside the shard buffers
    unit: int = -1      # stage 3: index of the unit it holds


@dataclasses.dataclass
class Unit:
    """Stage 3 gather unit: a module whose params are gathered/released together."""
    module: nn.Module
    index: int
    bucket: int = -1
    buf: torch.Tensor | None = None
    work: object = None
    state: int = _NONE


def _no_decay_names(model: nn.Module) -> set:
    out = set()
    for mname, mod in model.named_modules():
        cls = type(mod).__name__.lower()
        if "norm" in cls:
            for pname, _ in mod.named_parameters(recurse=False):
                out.add(f"{mname}.{pname}" if mname else pname)
    return out


def _is_cl(t: torch.Tensor) -> bool:
    return t.dim() == 4 and t.is_contiguous(memory_format=torch.channels_last) and not t.is_contiguous()


def _round_up(x: int, m: int) -> int:
    return (x + m - 1) // m * m


def find_units(model: nn.Module) -> list:
    """Stage-3 gather units in forward order: the root (params not inside a
    repeated block: embeddings, final norm, head -- used at both ends of the
    forward) first, then every element of every ``nn.ModuleList`` that owns
    trainable params (transformer / UNet blocks)."""
    blocks, claimed = [], set()
    for mod in model.modules():
        if isinstance(mod, nn.ModuleList):
            for child in mod:
                ps = [p for p in child.parameters() if p.requires_grad and id(p) not in claimed]
                if ps:
                    blocks.append(child)
                    claimed.update(id(p) for p in ps)
    return [model] + blocks


def param_consumers(model: nn.Module) -> list:
    """Forward-order modules that read the trainable params (stages 1-2 deferred all-gather): every
    element of every ``nn.ModuleList`` that owns params (a transformer block, read as a whole -- fused
    block paths take their sub-layers' weights directly), then each remaining module with direct
    params (embeddings, final norm, head -- each is called as a module where it is used)."""
    blocks = find_units(model)[1:]
    claimed = {id(p) for b in blocks for p in b.parameters()}
    # registration order stands in for forward order: modules registered before the first block
    # (embeddings) are read before it, the rest (final norm, LM head -- the largest bucket) after the
    # last block, so block 0's gathers are not queued behind the head's
    first = id(blocks[0]) if blocks else None
    before, after, seen_block = [], [], False
    for m in model.modules():
        if id(m) == first:
            seen_block = True
        if any(p.requires_grad and id(p) not in claimed for p in m.parameters(recurse=False)):
            (after if seen_block else before).append(m)
    return before + blocks + after


def _param_linear_forward(mod: nn.Linear, x):
    from ..ops.linear import param_linear
    return param_linear(x, mod.weight, mod.bias)


class TrainEngine:
    def __init__(self, model: nn.Module, lr: float = 5e-5, betas=(0.9, 0.999), eps: float = 1e-8,
                 weight_decay: float = 0.0, max_grad_norm: float = 1.0, zero_stage: int = 0,
                 grad_accum: int = 1, bucket_elems: int = int(2e8), group=None,
                 comm_dtype: torch.dtype = torch.float32, loss_scaler=None, optim_bits: int = 32,
                 offload_optimizer: bool = False, offload_param: bool = False, max_inflight: int = 3):
        self.model = model
        opt_cls = HostOffloadAdamW if offload_optimizer else (FlatAdamW8bit if optim_bits == 8 else FlatAdamW)
        self.group = group
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1
        self.rank = dist.get_rank(group) if dist.is_initialized() else 0
        if zero_stage not in (0, 1, 2, 3):
            raise ValueError(f"zero_stage must be 0..3, got {zero_stage}")
        self.zero_stage = zero_stage                       # requested (ds_config / CLI)
        self.stage = zero_stage if self.world > 1 else 0   # effective
        self.sharded = self.stage >= 1
        self.part_grads = self.stage >= 2
        self.part_params = self.stage >= 3
        self.grad_accum = max(1, grad_accum)
        self.max_grad_norm = max_grad_norm
        self.comm_dtype = comm_dtype
        self.loss_scaler = loss_scaler
        self.max_inflight = max(1, max_inflight)
        dev = next(model.parameters()).device
        self.device = dev
        self.dtype = next(model.parameters()).dtype
        if self.stage != zero_stage:
            log.info("ZeRO stage %d requested with world size 1: running as stage 0", zero_stage)

        no_decay = _no_decay_names(model)
        unit = ALIGN * self.world
        slots, buckets = [], []
        if self.part_params:
            # one bucket per gather unit, laid out in backward order (last block first, root last)
            self.units = [Unit(m, i) for i, m in enumerate(find_units(model))]
            owner = {}
            for u in reversed(self.units):  # blocks claim their params before the root
                for p in u.module.parameters():
                    if p.requires_grad and id(p) not in owner:
                        owner[id(p)] = u.index
            named = [(n, p) for n, p in model.named_parameters() if p.requires_grad]
            off = 0
            for u in list(reversed(self.units[1:])) + [self.units[0]]:
                mine = [(n, p) for n, p in reversed(named) if owner[id(p)] == u.index]
                if not mine:
                    continue
                bstart, cur = off, []
                for n, p in mine:
                    s = ParamSlot(n, p, off, p.numel(), not (n.endswith("bias") or n in no_decay), len(buckets),
                                  tuple(p.shape))
                    slots.append(s)
                    cur.append(s)
                    off = _round_up(off + p.numel(), ALIGN)
                size = _round_up(off - bstart, unit)
                u.bucket = len(buckets)
                buckets.append(Bucket(bstart, size, cur, unit=u.index))
                off = bstart + size
            self.units = [u for u in self.units if u.bucket >= 0]
            for i, u in enumerate(self.units):
                u.index = i
                buckets[u.bucket].unit = i
        else:
            self.units = []
            named = list(reversed([(n, p) for n, p in model.named_parameters() if p.requires_grad]))
            off, cur, bstart = 0, [], 0
            for n, p in named:
                s = ParamSlot(n, p, off, p.numel(), not (n.endswith("bias") or n in no_decay), len(buckets),
                              tuple(p.shape))
                slots.append(s)
                cur.append(s)
                off = _round_up(off + p.numel(), ALIGN)
                if off - bstart >= bucket_elems:
                    size = _round_up(off - bstart, unit)
                    buckets.append(Bucket(bstart, size, cur))
                    off = bstart + size
                    bstart, cur = off, []
            if cur:
                size = _round_up(off - bstart, unit)
                buckets.append(Bucket(bstart, size, cur))
                off = bstart + size
        self.total = off
        self.slots, self.buckets = slots, buckets
        self._by_param = {id(s.param): s for s in slots}

        # ---- decay mask per 64-block (full layout)
        full_mask = torch.zeros(self.total // ALIGN, dtype=torch.uint8)
        for s in slots:
            if s.decay:
                full_mask[s.offset // ALIGN:_round_up(s.offset + s.numel, ALIGN) // ALIGN] = 1

        # ---- parameters: flat bf16 buffer the model reads views of (stages 0-2)
        self.flat = None
        if not self.part_params:
            self.flat = torch.zeros(self.total, device=dev, dtype=self.dtype)
            with torch.no_grad():
                for s in slots:
                    view = self.flat[s.offset:s.offset + s.numel]
                    p = s.param.detach()
                    if _is_cl(p):
                        # channels-last conv weight (SD UNet on MI355X): keep the NHWC memory order in the
                        # flat buffer so MIOpen's NHWC kernels read it without a per-call layout copy
                        O, I, kh, kw = p.shape
                        view.copy_(p.permute(0, 2, 3, 1).reshape(-1))
                        s.param.data = view.view(O, kh, kw, I).permute(0, 3, 1, 2)
                    else:
                        view.copy_(p.reshape(-1))
                        s.param.data = view.view(s.param.shape)
        # ---- full fp32 gradient buffer (stages 0-1)
        self.grad = None if self.part_grads else torch.zeros(self.total, device=dev, dtype=torch.float32)

        # ---- optimizer shard
        self.shard_grad = self.shard_bf16 = None
        if self.sharded:
            shard = self.total // self.world
            self.shard_grad = torch.zeros(shard, device=dev, dtype=torch.float32)
            host_params = self.part_params and offload_param and offload_optimizer and dev.type == "cuda"
            self.shard_bf16 = torch.empty(shard, dtype=self.dtype, device="cpu" if host_params else dev,
                                          pin_memory=host_params)
            self.offload_param = host_params
            if offload_param and not host_params and self.rank == 0:
                log.info("offload_param honoured only with stage 3 + offload_optimizer on GPU; bf16 shard in HBM")
            master = torch.empty(shard, device=dev, dtype=torch.float32)
            mask = torch.empty(shard // ALIGN, dtype=torch.uint8)
            so = 0
            for bk in buckets:
                piece = bk.size // self.world
                bk.shard_off = so
                lo = bk.start + self.rank * piece
                master[so:so + piece].copy_(self._bucket_values(bk)[self.rank * piece:(self.rank + 1) * piece])
                mask[so // ALIGN:(so + piece) // ALIGN] = full_mask[lo // ALIGN:(lo + piece) // ALIGN]
                so += piece
            self.shard_bf16.copy_(master)
            self.opt = opt_cls(master, lr, betas, eps, weight_decay, mask.to(dev),
                               model_bf16=self.shard_bf16, grad=self.shard_grad)
        else:
            self.offload_param = False
            master = self.flat.float()
            self.opt = opt_cls(master, lr, betas, eps, weight_decay, full_mask.to(dev),
                               model_bf16=self.flat, grad=self.grad)

        # ---- stage 3: drop the full params, install gather/release hooks
        self._empty = torch.empty(0, device=dev, dtype=self.dtype)
        self._hold = 0
        self._in_bwd = False
        self._mod_hooks = []
        if self.part_params:
            for s in slots:
                s.param.data = self._empty
            for mod in model.modules():  # save the Parameter, not a transposed view, for backward
                if isinstance(mod, nn.Linear):
                    mod.forward = functools.partial(_param_linear_forward, mod)
            model._param_linear = True  # tied LM heads (CausalLM.logits_from_hidden)
            for u in self.units:
                m = u.module
                self._mod_hooks += [
                    m.register_forward_pre_hook(functools.partial(self._pre_fwd, u)),
                    m.register_forward_hook(functools.partial(self._post_fwd, u)),
                    m.register_full_backward_pre_hook(functools.partial(self._pre_bwd, u)),
                ]

        # ---- stages 1-2: deferred parameter all-gather. AdamW updates the rank's shard; instead of
        # gathering every bucket right after it (an exposed collective of all the bf16 params: ~12 GB
        # for GPT-J, tens of ms over xGMI at 8 ranks), step() launches the gathers asynchronously in
        # forward order and each consumer module's forward pre-hook makes the compute stream wait
        # for just its buckets (then re-derives its transposed weight copies): the next step's
        # forward runs under the remaining gathers. Models opt in (supports_deferred_param_gather);
        # state_dict() / publish() / sync_params() wait for everything. KCA_DEFER_ALLGATHER=0: off.
        import os as _os
        self._defer_ag = (self.sharded and not self.part_params and self.world > 1
                          and getattr(model, "supports_deferred_param_gather", False)
                          and _os.environ.get("KCA_DEFER_ALLGATHER", "1") not in ("0", "false"))
        self._ag_works: dict = {}
        self._consumers = []
        if self._defer_ag:
            for m in param_consumers(model):
                bs = sorted({self._by_param[id(p)].bucket for p in m.parameters() if id(p) in self._by_param})
                if bs:
                    self._consumers.append([m, bs, False])  # module, buckets, needs refresh
            for c in self._consumers:
                self._mod_hooks.append(c[0].register_forward_pre_hook(functools.partial(self._pre_consume, c)))
            self._mod_hooks.append(model.register_state_dict_pre_hook(lambda *a, **k: self.sync_params()))

        # ---- gradient hooks
        self._micro = 0
        self._works = []          # stages 0-1: (work, out, out_c)
        self._pending = []        # stages 2-3: (work, bucket, tmp, tmp_c, staging)
        self._staging = {}        # stages 2-3: bucket -> fp32 staging buffer (this micro-batch)
        self._shard_first = set()  # stages 2-3: buckets whose shard grads are written (not added) next
        self._bucket_done = [0] * len(buckets)
        self._bucket_launched = [False] * len(buckets)
        self._deferred = set()    # buckets launched in step() after the pre-reduce hooks
        self._touched = set()     # params with a grad this optimizer step
        self._seen = set()        # params with a grad this micro-batch
        self._pend = []           # small-gradient accumulations awaiting one batched launch
        self._pend_ids = set()    # their parameters (one entry per parameter per launch)
        self._stash = {}          # id(param) -> (dst, micro-batch-0 bf16 grad, scale): see _accum
        self._stash_bytes = 0     # bf16 bytes the stash holds (capped: _PAIR_ACCUM_MAX_BYTES)
        self._pre_reduce, self._pre_step = [], []
        self._norm_group, self._replicated, self._rep_ranges = None, {}, []
        self._hooks = [s.param.register_post_accumulate_grad_hook(self._hook) for s in slots]
        for s in slots:
            grad_sink.register(s.param, self._accum)
        self.native = dev.type == "cuda"
        # TN-layout backward GEMMs (ops/linear.py) for models that support them (they keep
        # full transposed weight copies, so not with partitioned params)
        import os
        if self.native and not self.part_params and os.environ.get("KCA_TN_GRADS", "1") not in ("0", "false") \
                and hasattr(model, "enable_tn_grads"):
            model.enable_tn_grads(True)

    # --------------------------------------------------------------- layout
    def _bucket_values(self, bk: Bucket) -> torch.Tensor:
        """Current bucket contents (flat-layout order, zero padding)."""
        if self.flat is not None:
            return self.flat[bk.start:bk.start + bk.size]
        out = torch.zeros(bk.size, device=self.device, dtype=self.dtype)
        for s in bk.slots:
            out[s.offset - bk.start:s.offset - bk.start + s.numel].copy_(s.param.detach().reshape(-1))
        return out

    def _piece(self, bk: Bucket):
        piece = bk.size // self.world
        return piece, bk.shard_off

    # ----------------------------------------------------- stage 3: params
    def _gather(self, u: Unit, wait: bool = True):
        if u.state == _NONE:
            bk = self.buckets[u.bucket]
            piece, so = self._piece(bk)
            src = self.shard_bf16[so:so + piece]
            if src.device != self.device:
                src = src.to(self.device, non_blocking=True)
            u.buf = torch.empty(bk.size, device=self.device, dtype=self.dtype)
            u.work = dist.all_gather_into_tensor(u.buf, src, group=self.group, async_op=True)
            u.state = _INFLIGHT
        if wait and u.state == _INFLIGHT:
            u.work.wait()
            u.work = None
            bk = self.buckets[u.bucket]
            for s in bk.slots:
                s.param.data = u.buf[s.offset - bk.start:s.offset - bk.start + s.numel].view(s.shape)
            u.state = _READY

    def _release(self, u: Unit):
        if u.state == _NONE or self._hold:
            return
        if u.state == _INFLIGHT:
            u.work.wait()
            u.work = None
        for s in self.buckets[u.bucket].slots:
            s.param.data = self._empty
        u.buf = None
        u.state = _NONE

    def _pre_fwd(self, u: Unit, mod, args):
        self._gather(u)
        if u.index + 1 < len(self.units):
            self._gather(self.units[u.index + 1], wait=False)  # prefetch the next block

    def _post_fwd(self, u: Unit, mod, args, out):
        if not self._in_bwd:  # (during backward this is an activation-checkpoint recompute)
            self._release(u)

    def _pre_bwd(self, u: Unit, mod, grad_out):
        self._gather(u)
        if u.index - 1 >= 1:
            self._gather(self.units[u.index - 1], wait=False)  # prefetch the previous block
        return None

    @contextlib.contextmanager
    def gathered(self):
        """Full parameters materialised on every rank for the duration (no-op
        below stage 3): checkpoint/final save (``stage3_gather_16bit_weights_
        on_model_save``), sampling, evaluation. All ranks must enter it.

        Stages 1-2 with deferred gathers: the last step's all-gathers finish first -- readers such as
        the decode engine take weights straight from sub-modules, so no block pre-hook would wait."""
        if not self.part_params:
            if self._defer_ag:
                self.sync_params()
            yield
            return
        for u in self.units:
            self._gather(u, wait=False)
        for u in self.units:
            self._gather(u)
        self._hold += 1
        try:
            yield
        finally:
            self._hold -= 1
            if not self._hold:
                for u in self.units:
                    self._release(u)

    # ------------------------------------------------------------------ hooks
    def _hook(self, p: torch.Tensor):
        g = p.grad
        if g is None:  # the op handed this gradient to the sink (autograd still fires the hook)
            return
        p.grad = None
        self._accum(p, g)

    def _dst(self, p: torch.Tensor):
        """(slot, fp32 destination of p's gradient this micro-batch, write-not-add, first micro-batch)."""
        s = self._by_param[id(p)]
        first_micro = id(p) not in self._seen
        # stages 0-1 accumulate across micro-batches in the full buffer; 2-3 start a fresh staging buffer
        first = first_micro if self.part_grads else id(p) not in self._touched
        if self.part_grads:
            bk = self.buckets[s.bucket]
            st = self._staging.get(s.bucket)
            if st is None:
                st = self._staging[s.bucket] = torch.zeros(bk.size, device=self.device, dtype=torch.float32)
            dst = st[s.offset - bk.start:s.offset - bk.start + s.numel]
        else:
            dst = self.grad[s.offset:s.offset + s.numel]
        return s, dst, first, first_micro

    def _accum(self, p: torch.Tensor, g: torch.Tensor):
        """Add one micro-batch gradient of ``p`` into fp32 storage (the full grad
        buffer, or the bucket's staging buffer under ZeRO-2/3) and launch the
        bucket's collective once the bucket is complete. Also the gradient sink
        (ops/grad_sink.py) that fused ops (ops/fused_block.py) call directly
        with row-strided column slices of a concatenated-weight dW."""
        s, dst, first, first_micro = self._dst(p)
        scale = 1.0 / self.grad_accum
        if g.dim() == 4 and _is_cl(p):  # flat slot holds the NHWC order
            g = g.permute(0, 2, 3, 1)
            g = g.reshape(-1) if g.is_contiguous() else g.contiguous().reshape(-1)
        small = ((self.native and g.dtype == torch.bfloat16 or _DEFER_CPU) and g.is_contiguous()
                 and s.numel <= _SMALL_GRAD and _MULTI_ACCUM
                 and not (g.is_cuda and torch.cuda.is_current_stream_capturing()))
        stashed = self._stash.get(id(p))
        if stashed is not None and (small or not (self.native and g.dtype == torch.bfloat16 and g.is_contiguous())
                                    or stashed[1].numel() != s.numel):
            # micro-batch 0's stashed gradient meets a micro-batch-1 gradient the pair kernel cannot take
            # (another branch below): land it first, so this one accumulates onto it (it used to
            # be overwritten by a later _land_stash)
            self._land(self._stash.pop(id(p)))
            self._stash_bytes -= stashed[1].numel() * 2
            first = False
        if small:
            # small gradients are batched into one kca_accum_grad_multi launch (flushed before any
            # bucket collective and at the end of backward); the entry keeps g alive until then
            # a parameter fed twice in one backward (a block applied twice: two sink calls) must not
            # have two entries in one launch -- their blocks would race on the same destination
            if id(p) in self._pend_ids:
                self._flush_small()
            self._pend.append((dst, g.reshape(-1), bool(first), scale))
            self._pend_ids.add(id(p))
            if len(self._pend) >= 256:
                self._flush_small()
        elif self.native and g.dtype == torch.bfloat16 and g.is_contiguous():
            st = self._stash.pop(id(p), None)
            if st is not None:
                self._stash_bytes -= st[1].numel() * 2
            if st is not None and st[1].numel() == s.numel:
                # micro-batch 1: both micro-batches' gradients into the buffer in one pass (8 instead of
                # 14 bytes per element; micro-batch 0 wrote nothing) -- bit-identical to the two passes
                _lib.call("kca_accum_grad_pair", dst.data_ptr(), st[1].data_ptr(), g.data_ptr(), scale, s.numel,
                          _lib.stream())
            else:
                if st is not None:  # (fed twice in micro-batch 0: the stashed one lands first)
                    self._land(st)
                    first = False
                if (_PAIR_ACCUM and first and first_micro and self._micro == 0 and self.grad_accum >= 2
                        and not self.part_grads and not torch.cuda.is_current_stream_capturing()
                        and self._stash_bytes + 2 * s.numel <= _PAIR_ACCUM_MAX_BYTES):
                    self._stash[id(p)] = (dst, g.reshape(-1), scale, s.bucket)  # lands with micro-batch 1's
                    self._stash_bytes += 2 * s.numel
                else:
                    _lib.call("kca_accum_grad", dst.data_ptr(), g.data_ptr(), scale, int(first), s.numel,
                              _lib.stream())
        elif (self.native and g.dtype == torch.bfloat16 and g.dim() == 2 and g.stride(1) == 1
              and g.shape[1] % 8 == 0 and g.stride(0) % 8 == 0 and g.data_ptr() % 16 == 0):
            _lib.call("kca_accum_grad_2d", dst.data_ptr(), g.data_ptr(), g.stride(0), g.shape[0], g.shape[1],
                      scale, int(first), _lib.stream())
        else:
            if first:
                dst.copy_(g.reshape(-1).float() * scale)
            else:
                dst.add_(g.reshape(-1).float(), alpha=scale)
        self._accounted(p, s, first_micro)

    def _accounted(self, p, s, first_micro: bool):
        """Bookkeeping after p's micro-batch gradient landed: launch its bucket's collective once every
        slot of the bucket has one."""
        self._touched.add(id(p))
        if first_micro:
            self._seen.add(id(p))
            if (self.part_grads or self._last_micro) and self.world > 1:
                self._bucket_done[s.bucket] += 1
                if self._bucket_done[s.bucket] == len(self.buckets[s.bucket].slots) \
                        and s.bucket not in self._deferred:
                    self._launch(s.bucket)

    def _flush_small(self):
        """One launch for the pending small-gradient accumulations (see _accum)."""
        pend, self._pend = self._pend, []
        self._pend_ids = set()
        if not pend:
            return
        if not self.native or _FLUSH_TORCH:  # CPU emulation of the batched path (tests of the engine logic)
            for dst, g, first, scale in pend:
                if first:
                    dst.copy_(g.float() * scale)
                else:
                    dst.add_(g.float(), alpha=scale)
            return
        import numpy as np
        by_scale: dict = {}
        for e in pend:
            by_scale.setdefault(e[3], []).append(e)
        for scale, es in by_scale.items():
            # the entries go to the kernel by value (kernel arguments), nothing on the device to manage
            tbl = np.array([[d.data_ptr(), g.data_ptr(), d.numel(), int(f)] for d, g, f, _ in es], dtype=np.int64)
            _lib.call("kca_accum_grad_multi", tbl.ctypes.data, len(es), float(scale), _lib.stream())
        # the gradient tensors are freed after the launch: the caching allocator only hands their
        # memory to work queued later on this stream

    def _land(self, st):
        dst, g, scale, _ = st
        _lib.call("kca_accum_grad", dst.data_ptr(), g.data_ptr(), scale, 1, g.numel(), _lib.stream())

    def _land_stash(self, bucket: int | None = None):
        """Stashed micro-batch-0 gradients whose parameter got none in micro-batch 1 (all of them
        before the optimizer; a bucket's before its collective reads the buffer): written as a first
        accumulation would have."""
        for k in [k for k, e in self._stash.items() if bucket is None or e[3] == bucket]:
            e = self._stash.pop(k)
            self._stash_bytes -= e[1].numel() * 2
            self._land(e)

    def _launch(self, bi: int):
        self._flush_small()
        self._land_stash(bi)
        if self._bucket_launched[bi]:
            return
        self._bucket_launched[bi] = True
        bk = self.buckets[bi]
        piece = bk.size // self.world
        if self.part_grads:
            st = self._staging.pop(bi, None)
            if st is None:  # no param of this bucket got a gradient in this micro-batch
                st = torch.zeros(bk.size, device=self.device, dtype=torch.float32)
            tmp = torch.empty(piece, device=self.device, dtype=torch.float32)
            if self.comm_dtype != torch.float32:
                src_c, tmp_c = st.to(self.comm_dtype), torch.empty(piece, device=self.device, dtype=self.comm_dtype)
                w = dist.reduce_scatter_tensor(tmp_c, src_c, group=self.group, async_op=True)
            else:
                tmp_c = None
                w = dist.reduce_scatter_tensor(tmp, st, group=self.group, async_op=True)
            self._pending.append((w, bi, tmp, tmp_c, st))
            if self.part_params and self._in_bwd:
                self._release(self.units[bk.unit])  # its backward is done: drop the gathered params
            while len(self._pending) > self.max_inflight:
                self._drain_one()
            return
        src = self.grad[bk.start:bk.start + bk.size]
        if self.sharded:
            out = self.shard_grad[bk.shard_off:bk.shard_off + piece]
            if self.comm_dtype != torch.float32:
                src_c = src.to(self.comm_dtype)
                out_c = torch.empty(piece, device=src.device, dtype=self.comm_dtype)
                w = dist.reduce_scatter_tensor(out_c, src_c, group=self.group, async_op=True)
                self._works.append((w, out, out_c))
            else:
                w = dist.reduce_scatter_tensor(out, src, group=self.group, async_op=True)
                self._works.append((w, None, None))
        else:
            w = dist.all_reduce(src, group=self.group, async_op=True)
            self._works.append((w, None, None))

    def _drain_one(self):
        w, bi, tmp, tmp_c, _st = self._pending.pop(0)
        w.wait()
        if tmp_c is not None:
            tmp.copy_(tmp_c)
        bk = self.buckets[bi]
        piece = bk.size // self.world
        out = self.shard_grad[bk.shard_off:bk.shard_off + piece]
        if bi in self._shard_first:
            out.copy_(tmp)
            self._shard_first.discard(bi)
        else:
            out.add_(tmp)

    def _end_micro(self):
        """Stages 2-3: every bucket is reduce-scattered once per micro-batch
        (buckets with a param that got no gradient are flushed here)."""
        self._seen = set()
        if self.part_grads and self.world > 1:
            for bi in range(len(self.buckets)):
                self._launch(bi)
            if self.part_params:
                for u in self.units:
                    self._release(u)
            self._bucket_done = [0] * len(self.buckets)
            self._bucket_launched = [False] * len(self.buckets)

    # -------------------------------------------------------------- training
    @property
    def _last_micro(self) -> bool:
        return self._micro == self.grad_accum - 1

    def _begin_micro(self):
        if self._micro == 0 and self.part_grads:
            self._shard_first = set(range(len(self.buckets)))

    def backward(self, loss: torch.Tensor):
        """Backward of one micro-batch (call grad_accum times, then step())."""
        if self.loss_scaler is not None and self.loss_scaler.enabled:
            loss = loss * self.loss_scaler.scale
        self._begin_micro()
        self._in_bwd = True
        try:
            loss.backward()
        finally:
            self._in_bwd = False
            self._flush_small()
        self._end_micro()
        self._micro += 1

    def backward_from(self, tensors, grads):
        """Backward of one micro-batch from an intermediate output (pipeline
        stages: ``tensors`` = this stage's output, ``grads`` = dL/d(output)
        received from the next stage; ``grads=None`` for a loss)."""
        self._begin_micro()
        self._in_bwd = True
        try:
            torch.autograd.backward(tensors, grads)
        finally:
            self._in_bwd = False
            self._flush_small()
        self._end_micro()
        self._micro += 1

    def add_pre_step(self, fn):
        """``fn(engine)`` runs after the gradient reduction, before clipping/AdamW."""
        self._pre_step.append(fn)

    def add_pre_reduce(self, fn, params=()):
        """``fn(engine)`` runs in ``step()`` on the full, not yet DP-reduced fp32
        gradients (e.g. summing a tied embedding's two pipeline-stage copies);
        the buckets holding ``params`` are held back from the overlapped launch
        until it ran. Needs the full gradient buffer (stages 0-1)."""
        if self.part_grads:
            raise NotImplementedError("pre-reduce gradient hooks need the full gradient buffer (ZeRO stage <= 1)")
        self._pre_reduce.append(fn)
        for p in params:
            self._deferred.add(self._by_param[id(p)].bucket)

    def slot_of(self, p) -> ParamSlot:
        return self._by_param[id(p)]

    def set_model_parallel(self, norm_group, replicated, copies: int = 1):
        """Tensor/pipeline parallel runs: the clip norm sums over ``norm_group``
        (all model-parallel shards of one replica). ``replicated``: names of
        params present ``copies`` times in that group (counted once), or a dict
        name -> copies (copies 0 = another rank counts it, e.g. the last
        stage's copy of a tied embedding)."""
        if self.part_params:
            raise NotImplementedError("ZeRO-3 with tensor/pipeline parallelism (use stage <= 2 over the DP group)")
        if not isinstance(replicated, dict):
            replicated = {n: copies for n in replicated}
        self._norm_group, self._replicated = norm_group, dict(replicated)
        # (lo, hi, weight) ranges in the optimizer's grad coordinates (full grad, or this rank's shard)
        rng = []
        for s in self.slots:
            c = self._replicated.get(s.name)
            if c is None or c == 1:
                continue
            w = 1.0 if c == 0 else (1.0 - 1.0 / c)
            if not self.sharded:
                rng.append((s.offset, s.offset + s.numel, w))
                continue
            bk = self.buckets[s.bucket]
            piece = bk.size // self.world
            plo = bk.start + self.rank * piece
            lo, hi = max(s.offset, plo), min(s.offset + s.numel, plo + piece)
            if lo < hi:
                rng.append((bk.shard_off + lo - plo, bk.shard_off + hi - plo, w))
        self._rep_ranges = rng

    def _replica_correction(self, sumsq: torch.Tensor) -> torch.Tensor:
        if not self._rep_ranges:
            return sumsq
        g = self.opt.grad
        adj = sumsq.clone()
        for lo, hi, w in self._rep_ranges:
            adj -= w * g[lo:hi].float().pow(2).sum()
        return adj

    def grad_norm(self) -> float:
        """Global L2 norm of the last step's (averaged, unscaled, pre-clip) gradient -- the value the
        clip used; equal across data-parallel layouts of the same global batch (one host sync)."""
        if getattr(self, "_gn", None) is None:
            return float("nan")
        sumsq, inv = self._gn
        return float(sumsq.float().sqrt() * inv)

    def step(self, lr: float | None = None) -> None:
        self._land_stash()
        if not self.part_grads:
            # grads of params that got no gradient this step are zero
            for s in self.slots:
                if id(s.param) not in self._touched:
                    self.grad[s.offset:s.offset + s.numel].zero_()
            for fn in self._pre_reduce:
                fn(self)
            if self.world > 1:
                for bi in range(len(self.buckets)):
                    self._launch(bi)
                for w, out, out_c in self._works:
                    w.wait()
                    if out is not None:
                        out.copy_(out_c)
        else:
            while self._pending:
                self._drain_one()
        for fn in self._pre_step:
            fn(self)
        inv = 1.0 / self.world
        if self.loss_scaler is not None and self.loss_scaler.enabled:
            inv /= self.loss_scaler.scale
        sumsq = self._replica_correction(self.opt.local_sumsq())
        if self.sharded:
            dist.all_reduce(sumsq, group=self.group)
        if self._norm_group is not None:
            dist.all_reduce(sumsq, group=self._norm_group)
        self._gn = (sumsq.detach().clone(), inv)
        self.opt.set_clip(sumsq, self.max_grad_norm, inv)
        self.opt.step(lr, use_clip=True)
        deferred = False
        if self.sharded and not self.part_params:
            if self._defer_ag:
                self._launch_param_gathers()
                deferred = True
            else:
                self._all_gather_params()
        if self.loss_scaler is not None and self.loss_scaler.enabled:
            self.loss_scaler.update(bool(self.opt.skipped.item()))
        self._refresh_derived(deferred=deferred)
        self._micro = 0
        self._works = []
        self._bucket_done = [0] * len(self.buckets)
        self._bucket_launched = [False] * len(self.buckets)
        self._touched = set()

    def _launch_param_gathers(self):
        """Every bucket's bf16 all-gather, async, in the consumers' forward order."""
        self.sync_params()  # (a previous step's gathers not consumed yet: finish them first)
        order, seen = [], set()
        for c in self._consumers:
            for b in c[1]:
                if b not in seen:
                    seen.add(b)
                    order.append(b)
        order += [b for b in range(len(self.buckets)) if b not in seen]
        for b in order:
            bk = self.buckets[b]
            piece = bk.size // self.world
            self._ag_works[b] = dist.all_gather_into_tensor(
                self.flat[bk.start:bk.start + bk.size], self.shard_bf16[bk.shard_off:bk.shard_off + piece],
                group=self.group, async_op=True)
        for c in self._consumers:
            c[2] = True

    def _pre_consume(self, c, module, args):
        if not c[2]:
            return None
        for b in c[1]:
            w = self._ag_works.pop(b, None)
            if w is not None:
                w.wait()  # the compute stream waits for this bucket's gather (no host block on RCCL)
        c[2] = False
        self._refresh_module(module)
        return None

    @staticmethod
    def _refresh_module(module):
        from ..ops.linear import TLinear
        for m in module.modules():
            if isinstance(m, TLinear):
                m.refresh_transposed()
        fused = getattr(module, "fused", None)
        if fused is not None and hasattr(fused, "refresh"):
            fused.refresh()

    def sync_params(self):
        """Finish every deferred parameter gather and re-derive what depends on the params."""
        if not self._ag_works and not any(c[2] for c in self._consumers):
            return
        for w in list(self._ag_works.values()):
            w.wait()
        self._ag_works.clear()
        for c in self._consumers:
            if c[2]:
                c[2] = False
                self._refresh_module(c[0])

    def _all_gather_params(self):
        ws = []
        for bk in self.buckets:
            piece = bk.size // self.world
            ws.append(dist.all_gather_into_tensor(
                self.flat[bk.start:bk.start + bk.size],
                self.shard_bf16[bk.shard_off:bk.shard_off + piece], group=self.group, async_op=True))
        for w in ws:
            w.wait()

    def train_batch(self, micro_batches, loss_fn, lr: float | None = None) -> torch.Tensor:
        """Run GAS micro-batches + optimizer step; returns the mean loss (device)."""
        assert len(micro_batches) == self.grad_accum
        total = None
        for mb in micro_batches:
            loss = loss_fn(mb)
            self.backward(loss)
            d = loss.detach().float()
            total = d if total is None else total + d
        self.step(lr)
        return total / self.grad_accum

    # ------------------------------------------------------------ state I/O
    def grad_norm(self) -> float:
        return float(self.opt.grad_norm.item())

    def layout_tag(self) -> str:
        """Hash of the flat layout (slot names/offsets, bucket bounds, param
        partitioning): stage 3 orders slots by gather unit, stages 0-2 by
        backward buckets, so equal totals do not imply equal layouts."""
        import hashlib
        h = hashlib.sha1(f"{int(self.part_params)}|{self.world}|{self.total}".encode())
        for s in self.slots:
            h.update(f"{s.name}:{s.offset}:{s.numel};".encode())
        for b in self.buckets:
            h.update(f"[{b.start}:{b.size}]".encode())
        return h.hexdigest()[:16]

    def optimizer_state(self) -> dict:
        return {"master": self.opt.master, **self.opt.state_dict(), "rank": self.rank,
                "world": self.world, "total": self.total, "zero_stage": self.stage,
                "requested_zero_stage": self.zero_stage, "layout": self.layout_tag()}

    def load_optimizer_state(self, sd: dict):
        if sd.get("world", 1) != self.world or sd.get("total") != self.total:
            raise ValueError("optimizer shard layout mismatch (world size or model changed)")
        if "layout" in sd and sd["layout"] != self.layout_tag():
            raise ValueError(f"optimizer state was saved with a different flat layout (ZeRO stage "
                             f"{sd.get('zero_stage')} vs {self.stage}, or bucket size / model changed); "
                             "resume with the same --zero-stage and bucket size")
        self.opt.master.copy_(sd["master"])
        self.opt.load_state_dict(sd)
        self.publish(self.opt.master)

    def _refresh_derived(self, deferred: bool = False):
        """Weights changed: re-derive per-model caches (transposed weight copies, UNet tables).
        ``deferred``: the params are still being gathered; each consumer re-derives its own copies
        in its forward pre-hook."""
        inv = getattr(self.model, "invalidate_weight_caches", None)
        if inv is not None:
            inv()
        if self.part_params or deferred:
            return
        fn = getattr(self.model, "refresh_transposed_weights", None)
        if fn is not None:
            fn()

    def publish(self, master_like: torch.Tensor):
        """Write bf16 model params from an fp32 tensor laid out like the
        optimizer master (the shard when ZeRO>=1), e.g. EMA weights for export."""
        self.sync_params()
        if self.sharded:
            self.shard_bf16.copy_(master_like)
            if not self.part_params:
                self._all_gather_params()
        else:
            self.flat.copy_(master_like)
        self._refresh_derived()

    def memory_report(self) -> dict:
        """Bytes this rank holds persistently per category."""
        b = lambda t: 0 if t is None else t.numel() * t.element_size()  # noqa: E731
        o = self.opt
        return {"zero_stage": self.stage, "params_bf16": b(self.flat) + b(self.shard_bf16) * (self.flat is None),
                "grads_fp32": b(self.grad) + b(self.shard_grad), "master_fp32": b(o.master),
                "optim_state": sum(b(getattr(o, k, None)) for k in ("exp_avg", "exp_avg_sq", "m_codes", "v_codes"))}

    def remove_hooks(self):
        for h in self._hooks + self._mod_hooks:
            h.remove()
        self._hooks, self._mod_hooks = [], []
        for s in self.slots:
            grad_sink.unregister(s.param)


__all__ = ["TrainEngine", "find_units"]
