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

Point-to-point traffic (``batch_isend_irecv`` of the pipeline stages and of
Adasum's recursive doubling, ``send`` / ``recv``) is staged the same way; the
``isend`` / ``irecv`` functions themselves stay the originals, because
``dist.P2POp`` accepts only those. ``parallel.dist.init_distributed`` enters
this mode for every entry point (trainers, servers) when the env var is set.

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
    """Completed ``Work`` stand-in for ``async_op=True`` callers (``get_future`` as DDP comm hooks
    use it: resolves to ``[result]``)."""

    def __init__(self, result=None):
        self._result = result

    def wait(self, *a, **k):
        return True

    def is_completed(self):
        return True

    def get_future(self):
        f = torch.futures.Future()
        f.set_result([self._result])
        return f


class _Recv:
    """A host-staged receive: ``wait`` completes the gloo receive, then copies into the device tensor."""

    def __init__(self, work, host, dst):
        self.work, self.host, self.dst = work, host, dst

    def wait(self, *a, **k):
        self.work.wait()
        self.dst.copy_(self.host)
        return True

    def is_completed(self):
        return self.work.is_completed()


class _Send:
    def __init__(self, work, host):
        self.work, self.host = work, host  # the host copy lives until the send completes

    def wait(self, *a, **k):
        return self.work.wait()

    def is_completed(self):
        return self.work.is_completed()


def _staged(t: torch.Tensor, force: bool) -> bool:
    return force or t.device.type != "cpu"


def install(force: bool = False):
    """Patch ``dist`` collectives to stage device tensors through host memory.
    ``force``: stage CPU tensors too (CPU tests of the staging logic)."""
    if _ORIG:
        return
    names = ("all_reduce", "reduce_scatter_tensor", "all_gather_into_tensor", "broadcast", "all_gather",
             "batch_isend_irecv", "send", "recv")
    for n in names:
        _ORIG[n] = getattr(dist, n)
    _ORIG["isend"], _ORIG["irecv"] = dist.isend, dist.irecv

    def _ret(async_op, result=None):
        return _Done(result) if async_op else None

    def all_reduce(tensor, op=dist.ReduceOp.SUM, group=None, async_op=False):
        if not _staged(tensor, force):
            return _ORIG["all_reduce"](tensor, op=op, group=group, async_op=async_op)
        h = tensor.detach().to("cpu", copy=True)
        _ORIG["all_reduce"](h, op=op, group=group)
        tensor.copy_(h)
        return _ret(async_op, tensor)

    def batch_isend_irecv(p2p_op_list):
        """Pipeline stage exchanges and Adasum pairs (parallel/pipeline.py, train/resnet.py): each
        op runs as its own gloo isend / irecv on a host copy; a receive lands in the device tensor
        when its work is waited on."""
        if not any(_staged(o.tensor, force) for o in p2p_op_list):
            return _ORIG["batch_isend_irecv"](p2p_op_list)
        works = []
        for o in p2p_op_list:
            tag = getattr(o, "tag", 0) or 0
            if o.op is _ORIG["isend"]:
                h = o.tensor.detach().to("cpu", copy=True).contiguous()
                works.append(_Send(_ORIG["isend"](h, o.peer, group=o.group, tag=tag), h))
            else:
                h = torch.empty(o.tensor.shape, dtype=o.tensor.dtype)
                works.append(_Recv(_ORIG["irecv"](h, o.peer, group=o.group, tag=tag), h, o.tensor))
        return works

    def send(tensor, dst=None, group=None, tag=0, **kw):
        if not _staged(tensor, force):
            return _ORIG["send"](tensor, dst, group=group, tag=tag, **kw)
        return _ORIG["send"](tensor.detach().to("cpu", copy=True).contiguous(), dst, group=group, tag=tag, **kw)

    def recv(tensor, src=None, group=None, tag=0, **kw):
        if not _staged(tensor, force):
            return _ORIG["recv"](tensor, src, group=group, tag=tag, **kw)
        h = torch.empty(tensor.shape, dtype=tensor.dtype)
        r = _ORIG["recv"](h, src, group=group, tag=tag, **kw)
        tensor.copy_(h)
        return r

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
                 ("all_gather", all_gather), ("batch_isend_irecv", batch_isend_irecv), ("send", send),
                 ("recv", recv)):
        setattr(dist, n, f)


def uninstall():
    for n, f in _ORIG.items():
        if n not in ("isend", "irecv"):  # never patched (P2POp only accepts the originals)
            setattr(dist, n, f)
    _ORIG.clear()


__all__ = ["ENV", "enabled", "install", "uninstall"]
