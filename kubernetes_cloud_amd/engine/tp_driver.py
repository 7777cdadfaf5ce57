"""Tensor-parallel serving driver: one engine, ``tp`` lock-stepped runners.

Rank 0 owns the scheduler (``LLMEngine``) and the HTTP front end; every call it
makes on its ``ModelRunner`` (prefill / sample_first / decode, and for beam
search decode_topk / copy_slots, and page release) is first published on a
control channel (``engine/ctrl_channel.py``: the native shared-memory ring when
the TP group shares a node -- no collective between decode steps -- else a gloo
broadcast), and follower ranks replay it on their own shard
(``follower_loop``). The GPU work of each call -- including the row-parallel
all-reduces and the vocab all-gather (the custom xGMI kernels for decode-size
messages, RCCL above) -- then runs in lock step. Sampling is replicated: identical gathered logits + identical
per-request seeds give identical tokens on every rank, so no token broadcast is
needed. This is the MI355X replacement for the DeepSpeed-Inference /
MII deployment of BLOOM-176B (bloom-176b-deepspeed, TP=8).
"""
from __future__ import annotations

import torch


def as_channel(ctrl):
    """A control channel (``send``/``recv``) or a process group (gloo broadcast)."""
    if getattr(ctrl, "kind", None) in ("shm", "gloo"):  # (a ProcessGroup has send/recv too)
        return ctrl
    from .ctrl_channel import GlooChannel
    return GlooChannel(ctrl)


class CollectiveRunner:
    # decode_async is mirrored too: rank 0 publishes step t+1 (rows chaining their input token from
    # step t on the device) before it reads step t, and the followers replay the same chain, so TP
    # decode gets the engine's one-step lookahead (the host's pickling / channel hop / scheduling
    # overlaps the GPU's step instead of sitting between steps)
    pipelined = True

    def __init__(self, runner, ctrl=None):
        self.runner = runner
        self.chan = as_channel(ctrl)

    def __getattr__(self, k):
        return getattr(self.runner, k)

    def _send(self, msg):
        self.chan.send(msg)

    def prefill(self, ids, slots, lens=None, start=None):
        self._send(("prefill", ids.to(torch.int32).numpy(), list(slots), lens, start))
        out = self.runner.prefill(ids, slots, lens, start)
        _check_ar()
        return out

    def sample_first(self, logits, rows):
        self._send(("sample_first", rows))
        return self.runner.sample_first(logits, rows)

    def decode(self, rows):
        self._send(("decode", rows))
        return self.runner.decode(rows)

    def decode_async(self, rows, prev=None):
        self._send(("decode_async", rows, prev is not None))
        return self.runner.decode_async(rows, prev=prev)

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


def follower_loop(runner, ctrl=None):
    """Ranks > 0: mirror rank 0's runner calls until it sends ``stop``."""
    chan = as_channel(ctrl)
    last_logits = None
    prev = older = None  # the last two decode_async handles (their chained tokens stay on the device)
    while True:
        obj = [chan.recv()]
        op = obj[0][0]
        if op == "stop":
            return
        if op == "prefill":
            last_logits = runner.prefill(torch.from_numpy(obj[0][1]).long(), obj[0][2], obj[0][3], obj[0][4])
            _check_ar()
        elif op == "sample_first":
            runner.sample_first(last_logits, obj[0][1])
        elif op == "decode":
            runner.decode(obj[0][1])
        elif op == "decode_async":
            # at most one step ahead of the GPU, as rank 0's engine (it reads step t before launching
            # t+2): step t+2 reuses step t's pinned upload / download buffers
            if older is not None and older.event is not None:
                older.event.synchronize()
            h = runner.decode_async(obj[0][1], prev=prev if obj[0][2] else None)
            older, prev = prev, h
        elif op == "decode_topk":
            runner.decode_topk(*obj[0][1:])
        elif op == "copy_slots":
            runner.copy_slots(*obj[0][1:])
        elif op == "release":
            runner.release(obj[0][1])
        else:
            raise RuntimeError(f"unknown op {op}")


__all__ = ["CollectiveRunner", "follower_loop"]
