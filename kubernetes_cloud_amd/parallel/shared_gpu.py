"""Shared-GPU rehearsal mode: N ranks on ONE GPU, collectives over gloo.

The driver's scaling bench runs ``bench.py --gpus N`` on a whole 8-GPU node;
the builder only ever gets a one-GPU box. RCCL refuses two ranks on one device
("duplicate GPU"), so to execute the exact N>1 code paths before that run
(ZeRO-1/2/3 bucketed reduce-scatter / all-gather, the TP decode engine with
its graph-captured xGMI all-reduce and all-gather, the gloo control plane),
``KCA_BENCH_SHARED_GPU=1`` makes every rank use ``cuda:0``, the default
process group gloo, and routes ``torch.distributed`` collectives on device
tensors through host copies (gloo's device paths do not cover every
collective the engine uses; the host path covers all of them). The custom xGMI kernels need no change: two processes
on one device map each other's IPC buffers the same way as two devices do.

Never used by production runs: everything here is a no-op unless
``install()`` is called, which only ``bench.py`` (under the env var) and the
GPU rehearsal tests do. Only the call sites that go through the ``dist``
module attribute (this package's engine, TP layers and drivers) are patched.
"""
from __future__ import annotations

import os

import torch
import torch.distributed as dist

ENV = "KCA_BENCH_SHARED_GPU"
_ORIG: dict = {}


def enabled() -> bool:
    return os.environ.get(ENV, "0") not in ("0", "", "false")


class _Done:
    """Completed ``Work`` stand-in for ``async_op=True`` callers."""

    def wait(self, *a, **k):
        return True

    def is_completed(self):
        return True


def _staged(t: torch.Tensor, force: bool) -> bool:
    return force or t.device.type != "cpu"


def install(force: bool = False):
    """Patch ``dist`` collectives to stage device tensors through host memory.
    ``force``: stage CPU tensors too (CPU tests of the staging logic)."""
    if _ORIG:
        return
    names = ("all_reduce", "reduce_scatter_tensor", "all_gather_into_tensor", "broadcast", "all_gather")
    for n in names:
        _ORIG[n] = getattr(dist, n)

    def _ret(async_op):
        return _Done() if async_op else None

    def all_reduce(tensor, op=dist.ReduceOp.SUM, group=None, async_op=False):
        if not _staged(tensor, force):
            return _ORIG["all_reduce"](tensor, op=op, group=group, async_op=async_op)
        h = tensor.detach().to("cpu", copy=True)
        _ORIG["all_reduce"](h, op=op, group=group)
        tensor.copy_(h)
        return _ret(async_op)

    def reduce_scatter_tensor(output, input, op=dist.ReduceOp.SUM, group=None, async_op=False):
        if not _staged(input, force):
            return _ORIG["reduce_scatter_tensor"](output, input, op=op, group=group, async_op=async_op)
        h = input.detach().to("cpu", copy=True).contiguous()
        o = torch.empty(output.shape, dtype=output.dtype)
        _ORIG["reduce_scatter_tensor"](o, h, op=op, group=group)
        output.copy_(o)
        return _ret(async_op)

    def all_gather_into_tensor(output, input, group=None, async_op=False):
        if not _staged(input, force):
            return _ORIG["all_gather_into_tensor"](output, input, group=group, async_op=async_op)
        w = dist.get_world_size(group)
        h = input.detach().to("cpu", copy=True).contiguous()
        parts = [torch.empty_like(h) for _ in range(w)]
        _ORIG["all_gather"](parts, h, group=group)
        output.copy_(torch.cat([p.view(-1) for p in parts]).view_as(output))
        return _ret(async_op)

    def broadcast(tensor, src, group=None, async_op=False):
        if not _staged(tensor, force):
            return _ORIG["broadcast"](tensor, src, group=group, async_op=async_op)
        h = tensor.detach().to("cpu", copy=True)
        _ORIG["broadcast"](h, src, group=group)
        tensor.copy_(h)
        return _ret(async_op)

    def all_gather(tensor_list, tensor, group=None, async_op=False):
        if not _staged(tensor, force):
            return _ORIG["all_gather"](tensor_list, tensor, group=group, async_op=async_op)
        h = tensor.detach().to("cpu", copy=True).contiguous()
        parts = [torch.empty_like(h) for _ in tensor_list]
        _ORIG["all_gather"](parts, h, group=group)
        for d, p in zip(tensor_list, parts):
            d.copy_(p)
        return _ret(async_op)

    for n, f in (("all_reduce", all_reduce), ("reduce_scatter_tensor", reduce_scatter_tensor),
                 ("all_gather_into_tensor", all_gather_into_tensor), ("broadcast", broadcast),
                 ("all_gather", all_gather)):
        setattr(dist, n, f)


def uninstall():
    for n, f in _ORIG.items():
        setattr(dist, n, f)
    _ORIG.clear()


__all__ = ["ENV", "enabled", "install", "uninstall"]
