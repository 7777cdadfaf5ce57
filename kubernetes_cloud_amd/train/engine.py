"""Training engine: flat parameters, fp32 grad accumulation, bucketed RCCL
reduce-scatter / all-reduce overlapped with the last backward, sharded
(ZeRO-1/2) fused AdamW, bf16 all-gather.

This is the MI355X-native replacement for the DeepSpeed ZeRO engine the
reference drives through HF Trainer (finetuner-workflow/finetuner/
ds_config.json:27-42: reduce_bucket_size 2e8, overlap_comm, reduce_scatter,
contiguous_gradients; finetuner.py:910-927 stage override) and for torch DDP /
Horovod in the kubeflow examples (resnet50_pytorch.py:121-122,
resnet50_horovod.py:136-140):

* every trainable parameter is re-pointed into ONE flat bf16 buffer (64-element
  aligned, ordered by reverse registration = backward order) -- the model's
  GEMMs read views of it;
* a post-accumulate-grad hook adds each bf16 grad into a flat fp32 buffer with
  the ``kca_accum_grad`` kernel (fp32 accumulation across micro-batches, as
  DeepSpeed does for 16-bit training) and frees the bf16 grad immediately;
* in the last micro-batch the hook launches the bucket's collective
  (reduce-scatter for ZeRO>=1, all-reduce for ZeRO-0) as soon as the bucket is
  complete, so communication overlaps the rest of the backward on RCCL's
  stream; buckets default to 2e8 elements like the reference's ds_config;
* each rank owns 1/W of every bucket (per-bucket sharding, so a bucket's
  reduce-scatter lands directly in the rank's contiguous optimizer shard);
  one ``kca_adamw`` launch updates the shard and writes its bf16 copy, which
  is all-gathered back into the flat buffer;
* grad clipping (global L2 norm) and the 1/W average are folded into one
  device scalar the AdamW kernel reads -- no host sync in the step.

ZeRO stage 3 (parameter partitioning) is accepted and runs as stage 2 on
MI355X: 288 GB HBM holds full bf16 replicas of every model the reference
trains on one node (GPT-J 12 GB, NeoX-20B 41 GB); optimizer state is what
gets sharded.
"""
from __future__ import annotations

import dataclasses
import math

import torch
import torch.distributed as dist
import torch.nn as nn

from ..ops import _lib, grad_sink
from .optim import FlatAdamW, FlatAdamW8bit, HostOffloadAdamW

ALIGN = 64


@dataclasses.dataclass
class ParamSlot:
    name: str
    param: nn.Parameter
    offset: int
    numel: int
    decay: bool
    bucket: int


@dataclasses.dataclass
class Bucket:
    start: int
    size: int
    slots: list
    shard_off: int = 0  # offset of this rank's piece inside the shard buffer


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


class TrainEngine:
    def __init__(self, model: nn.Module, lr: float = 5e-5, betas=(0.9, 0.999), eps: float = 1e-8,
                 weight_decay: float = 0.0, max_grad_norm: float = 1.0, zero_stage: int = 0,
                 grad_accum: int = 1, bucket_elems: int = int(2e8), group=None,
                 comm_dtype: torch.dtype = torch.float32, loss_scaler=None, optim_bits: int = 32,
                 offload_optimizer: bool = False):
        self.model = model
        opt_cls = HostOffloadAdamW if offload_optimizer else (FlatAdamW8bit if optim_bits == 8 else FlatAdamW)
        self.group = group
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1
        self.rank = dist.get_rank(group) if dist.is_initialized() else 0
        self.zero_stage = zero_stage
        self.sharded = zero_stage >= 1 and self.world > 1
        self.grad_accum = max(1, grad_accum)
        self.max_grad_norm = max_grad_norm
        self.comm_dtype = comm_dtype
        self.loss_scaler = loss_scaler
        dev = next(model.parameters()).device
        self.device = dev
        self.dtype = next(model.parameters()).dtype

        no_decay = _no_decay_names(model)
        named = [(n, p) for n, p in model.named_parameters() if p.requires_grad]
        named = list(reversed(named))  # ~backward order
        unit = ALIGN * self.world
        # ---- layout + buckets
        slots, buckets = [], []
        off = 0
        cur = []
        bstart = 0
        for n, p in named:
            decay = not (n.endswith("bias") or n in no_decay)
            s = ParamSlot(n, p, off, p.numel(), decay, len(buckets))
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

        # ---- flat bf16 params (model reads views of it)
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
        self.grad = torch.zeros(self.total, device=dev, dtype=torch.float32)

        # ---- decay mask per 64-block (full layout)
        full_mask = torch.zeros(self.total // ALIGN, dtype=torch.uint8)
        for s in slots:
            if s.decay:
                a = s.offset // ALIGN
                b = _round_up(s.offset + s.numel, ALIGN) // ALIGN
                full_mask[a:b] = 1

        # ---- optimizer shard
        if self.sharded:
            shard = self.total // self.world
            self.shard_grad = torch.empty(shard, device=dev, dtype=torch.float32)
            self.shard_bf16 = torch.empty(shard, device=dev, dtype=self.dtype)
            master = torch.empty(shard, device=dev, dtype=torch.float32)
            mask = torch.empty(shard // ALIGN, dtype=torch.uint8)
            so = 0
            for bk in buckets:
                piece = bk.size // self.world
                bk.shard_off = so
                lo = bk.start + self.rank * piece
                master[so:so + piece].copy_(self.flat[lo:lo + piece].float())
                mask[so // ALIGN:(so + piece) // ALIGN] = full_mask[lo // ALIGN:(lo + piece) // ALIGN]
                so += piece
            self.opt = opt_cls(master, lr, betas, eps, weight_decay, mask.to(dev),
                               model_bf16=self.shard_bf16, grad=self.shard_grad)
        else:
            master = self.flat.float()
            self.opt = opt_cls(master, lr, betas, eps, weight_decay, full_mask.to(dev),
                               model_bf16=self.flat, grad=self.grad)

        # ---- hooks
        self._micro = 0
        self._works = []
        self._bucket_done = [0] * len(buckets)
        self._bucket_launched = [False] * len(buckets)
        self._touched = set()
        self._hooks = [s.param.register_post_accumulate_grad_hook(self._hook) for s in slots]
        for s in slots:
            grad_sink.register(s.param, self._accum)
        self.native = dev.type == "cuda"
        # TN-layout backward GEMMs (ops/linear.py) for models that support them
        import os
        if self.native and os.environ.get("KCA_TN_GRADS", "1") not in ("0", "false") \
                and hasattr(model, "enable_tn_grads"):
            model.enable_tn_grads(True)

    # ------------------------------------------------------------------ hooks
    def _hook(self, p: torch.Tensor):
        g = p.grad
        if g is None:  # the op handed this gradient to the sink (autograd still fires the hook)
            return
        p.grad = None
        self._accum(p, g)

    def _accum(self, p: torch.Tensor, g: torch.Tensor):
        """Add one micro-batch gradient of ``p`` into the fp32 flat buffer and
        launch its bucket's collective once the bucket is complete. Also the
        gradient sink (ops/grad_sink.py) that fused ops (ops/fused_block.py) call
        directly with row-strided column slices of a concatenated-weight dW."""
        s = self._by_param[id(p)]
        dst = self.grad[s.offset:s.offset + s.numel]
        first = id(p) not in self._touched
        scale = 1.0 / self.grad_accum
        if g.dim() == 4 and _is_cl(p):  # flat slot holds the NHWC order
            g = g.permute(0, 2, 3, 1)
            g = g.reshape(-1) if g.is_contiguous() else g.contiguous().reshape(-1)
        if self.native and g.dtype == torch.bfloat16 and g.is_contiguous():
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
        self._touched.add(id(p))
        if self._last_micro and self.world > 1:
            self._bucket_done[s.bucket] += 1
            if self._bucket_done[s.bucket] == len(self.buckets[s.bucket].slots):
                self._launch(s.bucket)

    def _launch(self, bi: int):
        if self._bucket_launched[bi]:
            return
        self._bucket_launched[bi] = True
        bk = self.buckets[bi]
        src = self.grad[bk.start:bk.start + bk.size]
        if self.sharded:
            piece = bk.size // self.world
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

    # -------------------------------------------------------------- training
    @property
    def _last_micro(self) -> bool:
        return self._micro == self.grad_accum - 1

    def backward(self, loss: torch.Tensor):
        """Backward of one micro-batch (call grad_accum times, then step())."""
        if self.loss_scaler is not None and self.loss_scaler.enabled:
            loss = loss * self.loss_scaler.scale
        loss.backward()
        self._micro += 1

    def backward_from(self, tensors, grads):
        """Backward of one micro-batch from an intermediate output (pipeline
        stages: ``tensors`` = this stage's output, ``grads`` = dL/d(output)
        received from the next stage; ``grads=None`` for a loss)."""
        torch.autograd.backward(tensors, grads)
        self._micro += 1

    def add_pre_step(self, fn):
        """``fn(engine)`` runs after the gradient reduction, before clipping/AdamW."""
        if not hasattr(self, "_pre_step"):
            self._pre_step = []
        self._pre_step.append(fn)

    def set_model_parallel(self, norm_group, replicated, copies: int = 1):
        """Tensor/pipeline parallel runs: the clip norm sums over ``norm_group``
        (all model-parallel shards of one replica). ``replicated``: names of
        params present ``copies`` times in that group (counted once), or a dict
        name -> copies (copies 0 = another rank counts it, e.g. the last
        stage's copy of a tied embedding)."""
        if not isinstance(replicated, dict):
            replicated = {n: copies for n in replicated}
        self._norm_group, self._replicated = norm_group, dict(replicated)

    def _mp_sumsq(self, sumsq):
        grp = getattr(self, "_norm_group", None)
        if grp is None:
            return sumsq
        if self.sharded:
            raise NotImplementedError("model-parallel clipping with ZeRO sharding: use zero_stage=0 (plain DP)")
        adj = sumsq.clone()
        for sl in self.slots:
            c = self._replicated.get(sl.name)
            if c is not None and c != 1:
                w = 1.0 if c == 0 else (1.0 - 1.0 / c)
                adj -= w * self.grad[sl.offset:sl.offset + sl.numel].float().pow(2).sum()
        dist.all_reduce(adj, group=grp)
        return adj

    def step(self, lr: float | None = None) -> None:
        # grads of params that got no gradient this step are zero
        for s in self.slots:
            if id(s.param) not in self._touched:
                self.grad[s.offset:s.offset + s.numel].zero_()
        if self.world > 1:
            for bi in range(len(self.buckets)):
                self._launch(bi)
            for w, out, out_c in self._works:
                w.wait()
                if out is not None:
                    out.copy_(out_c)
        for fn in getattr(self, "_pre_step", ()):
            fn(self)
        inv = 1.0 / self.world
        if self.loss_scaler is not None and self.loss_scaler.enabled:
            inv /= self.loss_scaler.scale
        sumsq = self.opt.local_sumsq()
        if self.sharded:
            dist.all_reduce(sumsq, group=self.group)
        sumsq = self._mp_sumsq(sumsq)
        self.opt.set_clip(sumsq, self.max_grad_norm, inv)
        self.opt.step(lr, use_clip=True)
        if self.sharded:
            ws = []
            for bk in self.buckets:
                piece = bk.size // self.world
                ws.append(dist.all_gather_into_tensor(
                    self.flat[bk.start:bk.start + bk.size],
                    self.shard_bf16[bk.shard_off:bk.shard_off + piece], group=self.group,
                    async_op=True))
            for w in ws:
                w.wait()
        if self.loss_scaler is not None and self.loss_scaler.enabled:
            self.loss_scaler.update(bool(self.opt.skipped.item()))
        self._refresh_derived()
        self._micro = 0
        self._works = []
        self._bucket_done = [0] * len(self.buckets)
        self._bucket_launched = [False] * len(self.buckets)
        self._touched = set()

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

    def optimizer_state(self) -> dict:
        return {"master": self.opt.master, **self.opt.state_dict(), "rank": self.rank,
                "world": self.world, "total": self.total, "zero_stage": self.zero_stage}

    def load_optimizer_state(self, sd: dict):
        if sd.get("world", 1) != self.world or sd.get("total") != self.total:
            raise ValueError("optimizer shard layout mismatch (world size or model changed)")
        self.opt.master.copy_(sd["master"])
        self.opt.load_state_dict(sd)
        # refresh bf16 params from master
        if self.sharded:
            self.shard_bf16.copy_(self.opt.master)
            for bk in self.buckets:
                piece = bk.size // self.world
                dist.all_gather_into_tensor(self.flat[bk.start:bk.start + bk.size],
                                            self.shard_bf16[bk.shard_off:bk.shard_off + piece],
                                            group=self.group)
        else:
            self.flat.copy_(self.opt.master)
        self._refresh_derived()

    def _refresh_derived(self):
        """Weights changed: re-derive per-model caches (transposed weight copies)."""
        fn = getattr(self.model, "refresh_transposed_weights", None)
        if fn is not None:
            fn()

    def publish(self, master_like: torch.Tensor):
        """Write bf16 model params from an fp32 tensor laid out like the
        optimizer master (the shard when ZeRO>=1), e.g. EMA weights for export."""
        if self.sharded:
            self.shard_bf16.copy_(master_like)
            for bk in self.buckets:
                piece = bk.size // self.world
                dist.all_gather_into_tensor(self.flat[bk.start:bk.start + bk.size],
                                            self.shard_bf16[bk.shard_off:bk.shard_off + piece],
                                            group=self.group)
        else:
            self.flat.copy_(master_like)
        self._refresh_derived()

    def remove_hooks(self):
        for h in self._hooks:
            h.remove()
        self._hooks = []
        for s in self.slots:
            grad_sink.unregister(s.param)


def count_tokens_flops(cfg, seq: int) -> float:
    return cfg.flops_per_token(seq)


__all__ = ["TrainEngine", "math"]
