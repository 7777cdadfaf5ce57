"""Megatron-style tensor parallelism over RCCL/xGMI (SURVEY PAR-4, PAR-8, C12, C13).

Used by the BLOOM-176B TP=8 serving path (bloom-176b-deepspeed
02-inference-service.yaml:41, isvc-patch.txt:85-92 replaced DS-Inference's
kernel injection) and by TP training (the GPT-NeoX-20B job runs TP=2,
kubeflow/training-operator/gpt-neox/04-finetune-workflow.yaml:199-202).

Per transformer block, on each of ``tp`` ranks:
* fused QKV -> ``ColumnParallelLinear`` holding this rank's H/tp heads (q, k, v
  rows of those heads, so RoPE/attention/KV cache run unchanged on local heads);
* attention out-proj -> ``RowParallelLinear`` (input = local heads) + one
  all-reduce; bias added once after the reduce;
* MLP fc_in column-parallel (F/tp), fc_out row-parallel + one all-reduce;
* LayerNorms / embeddings replicated; the LM head is vocab-parallel
  (V/tp rows, a slice *view* of the tied embedding for BLOOM) followed by an
  all-gather of the logits.
So a token costs 2 all-reduces of [tokens, hidden] per layer -- at decode time
B x 14336 bf16 for BLOOM -- which RCCL runs over the point-to-point xGMI links;
TP degree is a launch choice (2/4/8), not baked into checkpoints.

Autograd: ``copy_to_tp`` (identity fwd / all-reduce bwd) feeds column-parallel
inputs, ``reduce_from_tp`` (all-reduce fwd / identity bwd) closes row-parallel
outputs, so the same modules train.

Loading: ``load_tp_model`` materialises one HF tensor at a time (lazy safetensors
reads through ``hf_to_native_plan``) and keeps only this rank's slice -- host
memory per rank stays at one tensor, not the 352 GB model.
"""
from __future__ import annotations

import glob
import json
import os

import torch
import torch.distributed as dist
import torch.nn as nn
import torch.nn.functional as F


# ------------------------------------------------------------- autograd
class _CopyToTP(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, group):
        ctx.group = group
        return x

    @staticmethod
    def backward(ctx, g):
        g = g.contiguous()
        dist.all_reduce(g, group=ctx.group)
        return g, None


class _ReduceFromTP(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, group):
        x = x.contiguous()
        dist.all_reduce(x, group=group)
        return x

    @staticmethod
    def backward(ctx, g):
        return g, None


class _GatherLastDim(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, group):
        ctx.group = group
        world = dist.get_world_size(group)
        x = x.contiguous()
        parts = [torch.empty_like(x) for _ in range(world)]
        dist.all_gather(parts, x, group=group)
        return torch.cat(parts, dim=-1)

    @staticmethod
    def backward(ctx, g):
        world = dist.get_world_size(ctx.group)
        rank = dist.get_rank(ctx.group)
        return g.chunk(world, dim=-1)[rank].contiguous(), None


def copy_to_tp(x, group):
    return _CopyToTP.apply(x, group) if torch.is_grad_enabled() and x.requires_grad else x


def reduce_from_tp(x, group):
    from .tp_emulation import is_emulated
    if is_emulated(group):  # one rank of a TP layout on one GPU (parallel/tp_emulation.py)
        return group.all_reduce_(x)
    if torch.is_grad_enabled() and x.requires_grad:
        return _ReduceFromTP.apply(x, group)
    x = x.contiguous()
    from .custom_ar import lookup
    ar = lookup(group)
    if ar is not None and ar.eligible(x):  # small decode messages: one-shot over xGMI peer memory
        return ar.all_reduce_(x)
    dist.all_reduce(x, group=group)
    return x


def gather_last_dim(x, group):
    from .tp_emulation import is_emulated
    if is_emulated(group):
        return group.all_gather_last(x)
    if torch.is_grad_enabled() and x.requires_grad:
        return _GatherLastDim.apply(x, group)
    return _gather_nograd(x, group)


_AR_GATHER = os.environ.get("KCA_AR_GATHER", "1") not in ("0", "false")


def _gather_nograd(x, group):
    world = dist.get_world_size(group)
    x = x.contiguous()
    from .custom_ar import lookup
    ar = lookup(group) if _AR_GATHER else None
    if ar is not None and ar.eligible(x):  # decode logits: one sync round over xGMI peer memory, graph-capturable
        flat = ar.all_gather(x)  # [world, *x.shape] flattened
        return flat.view(world, *x.shape).movedim(0, -2).reshape(*x.shape[:-1], world * x.shape[-1])
    parts = [torch.empty_like(x) for _ in range(world)]
    dist.all_gather(parts, x, group=group)
    return torch.cat(parts, dim=-1)


# --------------------------------------------------------------- layers
class ColumnParallelLinear(nn.Module):
    """y_local = x W_local^T (+ b_local); W_local: [out/tp, in]."""

    def __init__(self, in_features, out_local, bias, group):
        super().__init__()
        self.in_features, self.out_features = in_features, out_local
        self.weight = nn.Parameter(torch.empty(out_local, in_features))
        self.bias = nn.Parameter(torch.empty(out_local)) if bias else None
        self.group = group

    def forward(self, x):
        return F.linear(copy_to_tp(x, self.group), self.weight, self.bias)


class RowParallelLinear(nn.Module):
    """y = allreduce(x_local W_local^T) + b; W_local: [out, in/tp]."""

    def __init__(self, in_local, out_features, bias, group):
        super().__init__()
        self.in_features, self.out_features = in_local, out_features
        self.weight = nn.Parameter(torch.empty(out_features, in_local))
        self.bias = nn.Parameter(torch.empty(out_features)) if bias else None
        self.group = group

    def forward(self, x):
        y = reduce_from_tp(F.linear(x, self.weight), self.group)
        return y + self.bias if self.bias is not None else y


class ParallelLMHead(nn.Module):
    """Vocab-parallel head: local logits [.., V/tp] then all-gather -> [.., V]."""

    def __init__(self, hidden, v_local, bias, group, tied_to: nn.Embedding | None = None, rank: int = 0):
        super().__init__()
        self.group, self.v_local, self.rank = group, v_local, rank
        self._tied = [tied_to]  # plain list: not a registered submodule (no duplicate params)
        if tied_to is None:
            self.weight = nn.Parameter(torch.empty(v_local, hidden))
        self.bias = nn.Parameter(torch.empty(v_local)) if bias else None

    def local_weight(self):
        if self._tied[0] is not None:
            return self._tied[0].weight[self.rank * self.v_local:(self.rank + 1) * self.v_local]
        return self.weight

    def forward(self, y):
        logits = F.linear(copy_to_tp(y, self.group), self.local_weight(), self.bias)
        return gather_last_dim(logits, self.group)


# ---------------------------------------------------------- conversion
def tp_convert_(model, rank: int, world: int, group=None):
    """Swap a CausalLM's linears for TP shards (structure only; weights are
    uninitialised -- fill them with ``load_tp_state``)."""
    cfg = model.cfg
    H, D, d = cfg.n_heads, cfg.head_dim, cfg.hidden
    if H % world or cfg.ffn_dim % world or cfg.vocab_size % world:
        raise ValueError(f"heads {H}, ffn {cfg.ffn_dim}, vocab {cfg.vocab_size} must divide tp={world}")
    Hl, Fl, Vl = H // world, cfg.ffn_dim // world, cfg.vocab_size // world
    dev = next(model.parameters()).device
    dt = next(model.parameters()).dtype
    with torch.device(dev):
        _tp_swap(model, rank, group, H, D, d, Hl, Fl, Vl)
    if dev.type != "meta":
        model.to(dtype=dt)
    model.tp = (rank, world, group)
    return model


def _tp_swap(model, rank, group, H, D, d, Hl, Fl, Vl):
    for blk in model.h:
        at = blk.attn
        at.qkv = ColumnParallelLinear(d, 3 * Hl * D, at.qkv.bias is not None, group)
        at.out = RowParallelLinear(Hl * D, d, at.out.bias is not None, group)
        at.n_heads = Hl
        if at.alibi is not None:
            at.alibi = at.alibi[rank * Hl:(rank + 1) * Hl].clone()
        blk.mlp.fc_in = ColumnParallelLinear(d, Fl, blk.mlp.fc_in.bias is not None, group)
        blk.mlp.fc_out = RowParallelLinear(Fl, d, blk.mlp.fc_out.bias is not None, group)
    tied = model.lm_head is None
    model.lm_head = ParallelLMHead(d, Vl, (not tied) and model.lm_head.bias is not None, group,
                                   tied_to=model.wte if tied else None, rank=rank)
    if tied:
        # Tied embedding (BLOOM): the lookup grad is replicated on every rank, the
        # head grad lands only in this rank's vocab rows. Scale the lookup grad by
        # 1/tp and all-reduce the weight grad -> lookup + full head grad everywhere.
        world = dist.get_world_size(group) if dist.is_initialized() else 1
        model.wte.register_forward_hook(
            lambda mod, inp, out: _ScaleGrad.apply(out, 1.0 / world) if out.requires_grad else out)
        model.wte.weight.register_post_accumulate_grad_hook(
            lambda p: dist.all_reduce(p.grad, group=group))


class _ScaleGrad(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, s):
        ctx.s = s
        return x.view_as(x)

    @staticmethod
    def backward(ctx, g):
        return g * ctx.s, None


def shard_native_tensor(name: str, t: torch.Tensor, cfg, rank: int, world: int) -> torch.Tensor:
    """Slice a full native-layout tensor down to rank's TP shard."""
    H, D = cfg.n_heads, cfg.head_dim
    Hl = H // world
    if name.endswith("attn.qkv.weight") or name.endswith("attn.qkv.bias"):
        v = t.view(3, H, D, *t.shape[1:])[:, rank * Hl:(rank + 1) * Hl]
        return v.reshape(3 * Hl * D, *t.shape[1:]).contiguous()
    if name.endswith("attn.out.weight"):
        return t[:, rank * Hl * D:(rank + 1) * Hl * D].contiguous()
    if name.endswith("mlp.fc_in.weight") or name.endswith("mlp.fc_in.bias"):
        n = t.shape[0] // world
        return t[rank * n:(rank + 1) * n].contiguous()
    if name.endswith("mlp.fc_out.weight"):
        n = t.shape[1] // world
        return t[:, rank * n:(rank + 1) * n].contiguous()
    if name in ("lm_head.weight", "lm_head.bias"):
        n = t.shape[0] // world
        return t[rank * n:(rank + 1) * n].contiguous()
    return t  # replicated: LNs, embeddings, out/fc_out biases


@torch.no_grad()
def load_tp_state(model, plan: dict, rank: int, world: int):
    """Fill a ``tp_convert_``-ed model from a native-name -> producer plan."""
    cfg = model.cfg
    params = dict(model.named_parameters())
    seen = set()
    for name, produce in plan.items():
        if name not in params:
            continue
        full = produce()
        shard = shard_native_tensor(name, full, cfg, rank, world)
        p = params[name]
        if tuple(shard.shape) != tuple(p.shape):
            raise ValueError(f"{name}: shard {tuple(shard.shape)} != param {tuple(p.shape)}")
        p.copy_(shard.to(p.dtype))
        seen.add(name)
        del full, shard
    missing = [n for n in params if n not in seen]
    if missing:
        raise RuntimeError(f"TP load: missing {missing[:8]}")


class _LazySafetensors:
    """Mapping over one HF checkpoint dir that reads tensors on access."""

    def __init__(self, path: str):
        from safetensors import safe_open
        idx = os.path.join(path, "model.safetensors.index.json")
        if os.path.exists(idx):
            with open(idx) as f:
                wm = json.load(f)["weight_map"]
            files = sorted(set(wm.values()))
        else:
            files = [os.path.basename(p) for p in glob.glob(os.path.join(path, "*.safetensors"))]
            wm = None
        self.handles = {fn: safe_open(os.path.join(path, fn), framework="pt") for fn in files}
        self.where = {}
        for fn, h in self.handles.items():
            for k in h.keys():
                self.where[k] = fn
        if wm:
            self.where.update(wm)

    def __contains__(self, k):
        return k in self.where

    def __getitem__(self, k):
        return self.handles[self.where[k]].get_tensor(k)

    def keys(self):
        return self.where.keys()


def load_tp_model(path: str, rank: int, world: int, group=None, device=None, dtype=torch.bfloat16,
                  random_init: bool = False):
    """Build this rank's TP shard of the HF checkpoint at ``path``."""
    from ..models.causal_lm import CausalLM, alibi_slopes
    from ..models.config import LMConfig
    from ..models.hf_convert import hf_to_native_plan, prefixed_getter
    cfg = LMConfig.from_pretrained(path) if isinstance(path, str) else path
    with torch.device("meta"):
        m = CausalLM(cfg)
    tp_convert_(m, rank, world, group)
    # cast on meta first: materialising fp32 and then casting would peak at 3x the shard
    m = m.to(dtype).to_empty(device=device or "cpu")
    if cfg.alibi:
        Hl = cfg.n_heads // world
        for blk in m.h:
            blk.attn.alibi = alibi_slopes(cfg.n_heads)[rank * Hl:(rank + 1) * Hl].to(m.wte.weight.device)
    if random_init:
        g = torch.Generator(device=m.wte.weight.device).manual_seed(1234 + rank)
        with torch.no_grad():  # device-side init: a 176B/8 shard never touches host memory
            for n, p in m.named_parameters():
                if p.dim() >= 2:
                    p.normal_(0.0, 0.02, generator=g)
                else:
                    p.fill_(1.0 if n.endswith("weight") else 0.0)
        return m
    sd = _LazySafetensors(path)
    load_tp_state(m, hf_to_native_plan(cfg, prefixed_getter(sd), tuple(sd.keys())), rank, world)
    return m


def shard_model_from_full(full_model, rank: int, world: int, group=None):
    """TP shard built from an in-memory unsharded model (tests, small models)."""
    import copy
    sd = {k: v for k, v in full_model.state_dict().items()}
    m = copy.deepcopy(full_model)
    tp_convert_(m, rank, world, group)
    load_tp_state(m, {k: (lambda v=v: v) for k, v in sd.items()}, rank, world)
    return m


__all__ = ["ColumnParallelLinear", "RowParallelLinear", "ParallelLMHead", "tp_convert_", "load_tp_state",
           "load_tp_model", "shard_model_from_full", "shard_native_tensor", "copy_to_tp", "reduce_from_tp",
           "gather_last_dim"]
