"""Tensor-parallel serving driver: one engine, ``tp`` lock-stepped runners.

Rank 0 owns the scheduler (``LLMEngine``) and the HTTP front end; every call it
makes on its ``ModelRunner`` (prefill / sample_first / decode, and for beam
search decode_topk / copy_slots, and page release) is first
broadcast on a small CPU (gloo) control group, and follower ranks replay it on
their own shard (``follower_loop``). The GPU work of each call -- including the
row-parallel all-reduces and the vocab all-gather -- then runs in lock step
over RCCL. Sampling is replicated: identical gathered logits + identical
per-request seeds give identical tokens on every rank, so no token broadcast is
needed. This is the MI355X replacement for the DeepSpeed-Inference /
MII deployment of BLOOM-176B (bloom-176b-deepspeed, TP=8).
"""
from __future__ import annotations

import torch
import torch.distributed as dist


class CollectiveRunner:
    def __init__(self, runner, ctrl_group=None):
        self.runner, self.group = runner, ctrl_group

    def __getattr__(self, k):
        return getattr(self.runner, k)

    def _send(self, msg):
        obj = [msg]
        dist.broadcast_object_list(obj, src=0, group=self.group)

    def prefill(self, ids, slots, lens=None):
        self._send(("prefill", ids.tolist(), list(slots), lens))
        out = self.runner.prefill(ids, slots, lens)
        _check_ar()
        return out

    def sample_first(self, logits, rows):
        self._send(("sample_first", rows))
        return self.runner.sample_first(logits, rows)

    def decode(self, rows):
        self._send(("decode", rows))
        return self.runner.decode(rows)

    # beam search (engine.beam): scoring pass, cache re-order, and page release in lock step
    def decode_topk(self, tokens, positions, slots, k):
        self._send(("decode_topk", list(tokens), list(positions), list(slots), int(k)))
        return self.runner.decode_topk(tokens, positions, slots, k)

    def copy_slots(self, dst, src, upto):
        self._send(("copy_slots", list(dst), list(src), int(upto)))
        return self.runner.copy_slots(dst, src, upto)

    def release(self, slot):
        self._send(("release", int(slot)))
        return self.runner.release(slot)

    def shutdown(self):
        self._send(("stop",))


def _check_ar():
    """A timed-out xGMI all-reduce NaN-poisons its output and flags; surface it
    as an exception once per prefill (one device sync per request batch)."""
    from ..parallel.custom_ar import check_all
    check_all()


def follower_loop(runner, ctrl_group=None):
    """Ranks > 0: mirror rank 0's runner calls until it sends ``stop``."""
    last_logits = None
    while True:
        obj = [None]
        dist.broadcast_object_list(obj, src=0, group=ctrl_group)
        op = obj[0][0]
        if op == "stop":
            return
        if op == "prefill":
            last_logits = runner.prefill(torch.tensor(obj[0][1], dtype=torch.long), obj[0][2], obj[0][3])
            _check_ar()
        elif op == "sample_first":
            runner.sample_first(last_logits, obj[0][1])
        elif op == "decode":
            runner.decode(obj[0][1])
        elif op == "decode_topk":
            runner.decode_topk(*obj[0][1:])
        elif op == "copy_slots":
            runner.copy_slots(*obj[0][1:])
        elif op == "release":
            runner.release(obj[0][1])
        else:
            raise RuntimeError(f"unknown op {op}")


__all__ = ["CollectiveRunner", "follower_loop"]
