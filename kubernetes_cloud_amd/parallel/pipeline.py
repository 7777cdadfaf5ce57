"""Pipeline parallelism: stage partitioning + 1F1B schedule over RCCL p2p
(SURVEY PAR-5; the reference's GPT-NeoX-20B job runs PP=4 x TP=2 x DP=2,
kubeflow/training-operator/gpt-neox/04-finetune-workflow.yaml:199-202,
micro-batch 8 x GAS 96 :63-69,247-249).

``build_stage`` cuts a CausalLM into contiguous layer ranges (embedding on the
first stage, final LayerNorm + LM head + loss on the last); each stage's linear
layers can additionally be tensor-parallel (``tensor_parallel.tp_convert_``).
Stage boundaries carry one [micro_batch, seq, hidden] activation: the block's
pending residual branches are folded into the residual stream before the send.

``one_f_one_b`` runs PipeDream-flush 1F1B: ``P - s - 1`` warm-up forwards,
steady-state alternating forward/backward, cool-down backwards -- at most
``P - s`` activations alive per stage. Sends and receives are posted as one
``batch_isend_irecv`` per exchange so neighbouring stages never deadlock on
RCCL's rendezvous semantics, and the received gradient of micro-batch i feeds
the engine's backward directly (grad accumulation in fp32 via TrainEngine's
hooks; the DP reduction of the last micro-batch overlaps its backward).
"""
from __future__ import annotations

from collections import deque

import torch
import torch.distributed as dist
import torch.nn as nn
from torch.utils.checkpoint import checkpoint

from .. import ops


class PipelineStage(nn.Module):
    def __init__(self, full, lo: int, hi: int, first: bool, last: bool):
        super().__init__()
        self.cfg = full.cfg
        self.first, self.last = first, last
        self.lo, self.hi = lo, hi
        if first:
            self.wte = full.wte
            self.wpe = full.wpe
            self.emb_ln = full.emb_ln
            self.embed_scale = full.cfg.embed_scale
        self.h = nn.ModuleList(list(full.h)[lo:hi])
        if last:
            self.ln_f = full.ln_f
            self.lm_head = full.lm_head
            if full.lm_head is None:  # tied: last stage keeps its own copy, grads synced with stage 0
                self.head_weight = nn.Parameter(full.wte.weight.detach().clone()) if not first else None
        self.gradient_checkpointing = False

    def forward(self, x, labels=None):
        if self.first:
            h = self.wte(x)
            if self.embed_scale != 1.0:
                h = h * self.embed_scale
            if self.wpe is not None:
                h = h + self.wpe(torch.arange(x.shape[1], device=x.device)).to(h.dtype)
            if self.emb_ln is not None:
                h = self.emb_ln(h)
        else:
            h = x
        pending = ()
        for blk in self.h:
            if self.gradient_checkpointing and self.training and torch.is_grad_enabled():
                out = checkpoint(blk, h, None, *pending, use_reentrant=False)
            else:
                out = blk(h, None, *pending)
            h, pending = out[0], tuple(out[1:])
        if not self.last:
            for p in pending:
                h = h + p
            return h
        y, _ = self.ln_f(h, residual=pending) if pending else (self.ln_f(h), None)
        if self.lm_head is not None:
            logits = self.lm_head(y)
        else:
            w = self.wte.weight if self.first else self.head_weight
            logits = torch.nn.functional.linear(y, w)
        B, S = labels.shape
        shifted = torch.full_like(labels, -100)
        shifted[:, :-1] = labels[:, 1:]
        return ops.cross_entropy(logits.reshape(B * S, -1).contiguous(), shifted.view(-1), ignore_index=-100)


def split_layers(n_layers: int, pp: int) -> list[tuple[int, int]]:
    base, extra = divmod(n_layers, pp)
    out, lo = [], 0
    for s in range(pp):
        hi = lo + base + (1 if s < extra else 0)
        out.append((lo, hi))
        lo = hi
    return out


def build_stage(full, stage: int, pp: int) -> PipelineStage:
    lo, hi = split_layers(full.cfg.n_layers, pp)[stage]
    return PipelineStage(full, lo, hi, stage == 0, stage == pp - 1)


class P2P:
    """Point-to-point exchanges with the neighbouring stages (global ranks)."""

    def __init__(self, prev_rank: int | None, next_rank: int | None, shape, dtype, device):
        self.prev, self.next = prev_rank, next_rank
        self.shape, self.dtype, self.device = shape, dtype, device

    def _run(self, ops_):
        if not ops_:
            return
        for w in dist.batch_isend_irecv(ops_):
            w.wait()

    def _buf(self):
        return torch.empty(self.shape, dtype=self.dtype, device=self.device)

    def recv_forward(self):
        b = self._buf()
        self._run([dist.P2POp(dist.irecv, b, self.prev)])
        return b

    def send_forward(self, y):
        self._run([dist.P2POp(dist.isend, y.detach().contiguous(), self.next)])

    def recv_backward(self):
        b = self._buf()
        self._run([dist.P2POp(dist.irecv, b, self.next)])
        return b

    def send_backward(self, dx):
        self._run([dist.P2POp(dist.isend, dx.contiguous(), self.prev)])

    def send_forward_recv_backward(self, y):
        b = self._buf()
        self._run([dist.P2POp(dist.isend, y.detach().contiguous(), self.next), dist.P2POp(dist.irecv, b, self.next)])
        return b

    def send_backward_recv_forward(self, dx):
        b = self._buf()
        self._run([dist.P2POp(dist.isend, dx.contiguous(), self.prev), dist.P2POp(dist.irecv, b, self.prev)])
        return b


def one_f_one_b(stage: PipelineStage, engine, p2p: P2P, micro_batches: list, stage_idx: int, pp: int):
    """One optimizer step's worth of micro-batches through the pipeline.
    ``micro_batches``: token tensors [mb, S] (used by the first stage as input
    and by the last as labels). Returns the summed loss on the last stage."""
    M = len(micro_batches)
    first, last = stage_idx == 0, stage_idx == pp - 1
    warm = min(pp - stage_idx - 1, M)
    live = deque()
    loss_sum = torch.zeros((), device=p2p.device)

    def fwd(i, x):
        if first:
            inp = micro_batches[i]
        else:
            inp = x.requires_grad_(True)
        out = stage(inp, labels=micro_batches[i] if last else None)
        if last:
            nonlocal loss_sum
            loss_sum = loss_sum + out.detach().float()  # engine's hooks average over grad_accum
        return inp, out

    def bwd(inp, out, dy):
        engine.backward_from(out, None if last else dy)
        return None if first else inp.grad

    x = None
    for i in range(warm):
        x = None if first else p2p.recv_forward()
        inp, out = fwd(i, x)
        if not last:
            p2p.send_forward(out)
        live.append((inp, out))
    rem = M - warm
    if rem > 0 and not first:
        x = p2p.recv_forward()
    for j in range(rem):
        i = warm + j
        inp, out = fwd(i, x)
        dy = None if last else p2p.send_forward_recv_backward(out)
        live.append((inp, out))
        inp0, out0 = live.popleft()
        dx = bwd(inp0, out0, dy)
        if first:
            continue
        if j == rem - 1:
            p2p.send_backward(dx)
        else:
            x = p2p.send_backward_recv_forward(dx)
    for _ in range(warm):
        inp0, out0 = live.popleft()
        dy = None if last else p2p.recv_backward()
        dx = bwd(inp0, out0, dy)
        if not first:
            p2p.send_backward(dx)
    return loss_sum


def tie_embedding_grads(engine, stage: PipelineStage, group):
    """Tied input/output embedding split across the first and last stage: each
    keeps a copy; their fp32 grads are summed over ``group`` once per step,
    after the pipeline flush (a per-micro-batch collective inside backward
    would deadlock the 1F1B schedule) and before the optimizer."""
    if group is None:
        return
    p = stage.wte.weight if stage.first else getattr(stage, "head_weight", None)
    if p is None:
        return
    slot = engine.slot_of(p)

    def fn(eng):
        # on the full local grads, before the DP reduction (sums commute); the
        # slot's bucket is held back from the overlapped launch until this ran
        dist.all_reduce(eng.grad[slot.offset:slot.offset + slot.numel], group=group)
    engine.add_pre_reduce(fn, params=(p,))


__all__ = ["PipelineStage", "build_stage", "split_layers", "P2P", "one_f_one_b", "tie_embedding_grads"]
