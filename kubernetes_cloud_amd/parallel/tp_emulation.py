"""Rank-local emulation of one tensor-parallel rank on a single GPU.

BASELINE config 4 serves BLOOM-176B at TP=8 (online-inference/bloom-176b-deepspeed/
02-inference-service.yaml:41; files/isvc-patch.txt:85-89). One rank of that layout holds
1/8 of every projection -- QKV 14336 -> 5376, out-proj 1792 -> 14336, fc_in 14336 -> 7168,
fc_out 7168 -> 14336 -- plus a 31,360-row vocab shard of the head: ~44 GB, which one
288 GB MI355X holds. Its decode step is a different kernel mix from a full-width layer
(each projection streams 51-205 MB, ~8-34 us, so launch ramps and tails weigh far more).

``EmulatedTPGroup(world, rank)`` stands in for the rank's process group: the TP modules
(``parallel.tensor_parallel``) are built with exactly the shapes rank ``rank`` of a
``world``-way run holds, and the collectives become local stand-ins:

* all-reduce: identity (each rank's partial sum is taken as the sum). ``allreduce_calls``
  counts them so the report can price them separately (a real run adds one xGMI
  all-reduce of B x hidden bf16 per row-parallel projection);
* all-gather of the vocab-parallel logits: the local shard tiled ``world`` times (same
  output shape, so the sampler runs over the full vocabulary).

Tokens produced this way are not those of the full model (the weights are random anyway);
what the emulation measures is the per-rank HBM stream and kernel schedule.
"""
from __future__ import annotations

import torch


class EmulatedTPGroup:
    def __init__(self, world: int, rank: int = 0):
        if world < 1 or not 0 <= rank < world:
            raise ValueError(f"rank {rank} of world {world}")
        self.world, self.rank = world, rank
        self.allreduce_calls = 0
        self.allgather_calls = 0

    def size(self) -> int:
        return self.world

    def all_reduce_(self, x: torch.Tensor) -> torch.Tensor:
        self.allreduce_calls += 1
        return x

    def all_gather_last(self, x: torch.Tensor) -> torch.Tensor:
        self.allgather_calls += 1
        n = x.shape[-1]
        return x.unsqueeze(-2).expand(*x.shape[:-1], self.world, n).reshape(*x.shape[:-1], self.world * n)

    def __repr__(self):
        return f"EmulatedTPGroup(rank={self.rank}, world={self.world})"


def is_emulated(group) -> bool:
    return isinstance(group, EmulatedTPGroup)


def emulated_rank_model(cfg, world: int, rank: int = 0, device=None, dtype=torch.bfloat16):
    """Rank ``rank``'s random-init TP shard of ``cfg`` with emulated collectives."""
    from .tensor_parallel import load_tp_model
    return load_tp_model(cfg, rank, world, EmulatedTPGroup(world, rank), device=device, dtype=dtype,
                         random_init=True)


__all__ = ["EmulatedTPGroup", "is_emulated", "emulated_rank_model"]
