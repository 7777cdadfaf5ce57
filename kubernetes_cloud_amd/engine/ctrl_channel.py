"""Control-plane channels of the tensor-parallel serving engine.

Rank 0 publishes every runner call (``tp_driver.CollectiveRunner``) and the
follower ranks replay it (``tp_driver.follower_loop``). Two transports:

* ``ShmChannel`` -- the native single-producer / multi-consumer ring in POSIX
  shared memory (``csrc/runtime/ctrl_channel.cpp``), used when every rank of
  the TP group runs on one node (TP always stays inside an xGMI node): a decode
  step costs rank 0 one pickle + memcpy, and a follower spinning on the ring
  picks it up within microseconds. No collective sits between decode steps.
* ``GlooChannel`` -- ``broadcast_object_list`` on a CPU (gloo) group, for
  groups that span hosts or when the native library is unavailable.

``open_channel(group)`` picks one collectively (one gloo exchange at setup).
"""
from __future__ import annotations

import ctypes
import os
import pickle
import socket
import uuid

import torch.distributed as dist


class ChannelError(RuntimeError):
    pass


class GlooChannel:
    kind = "gloo"

    def __init__(self, group=None, src: int = 0):
        self.group, self.src = group, src

    def send(self, msg):
        dist.broadcast_object_list([msg], src=self.src, group=self.group)

    def recv(self):
        obj = [None]
        dist.broadcast_object_list(obj, src=self.src, group=self.group)
        return obj[0]

    def close(self):
        pass


class ShmChannel:
    """One writer (``reader=-1``) or reader ``reader`` of a named shm ring."""

    kind = "shm"

    def __init__(self, name: str, reader: int, readers: int = 0, slots: int = 16, slot_bytes: int = 1 << 20,
                 timeout_s: float | None = None):
        """``timeout_s``: bound on a send waiting for a stalled reader and on a
        recv waiting for the writer; None = a reader waits as long as the
        writer lives (an idle server), a writer 600 s."""
        from ..io import native
        self._lib = native.load()
        self.name, self.reader = name, reader
        self.block = timeout_s is None
        self.timeout_ms = int((600.0 if timeout_s is None else timeout_s) * 1000)
        if reader < 0:
            self._h = self._lib.kca_chan_create(name.encode(), slots, slot_bytes, readers)
        else:
            self._h = self._lib.kca_chan_open(name.encode(), 120_000 if self.block else self.timeout_ms)
        if not self._h:
            raise ChannelError(f"shm channel {name!r}: {'create' if reader < 0 else 'open'} failed")
        n = self._lib.kca_chan_slot_bytes(self._h)
        self._buf = ctypes.create_string_buffer(n)
        self._cap = n
        self.sent = 0

    def send(self, msg):
        data = pickle.dumps(msg, protocol=pickle.HIGHEST_PROTOCOL)
        rc = self._lib.kca_chan_send(self._h, data, len(data), self.timeout_ms)
        if rc != 0:
            raise ChannelError(f"shm channel send failed ({rc}: {'reader stalled' if rc == -2 else 'closed'})")
        self.sent += 1

    def recv(self):
        parts = []
        last = ctypes.c_int(0)
        while True:
            n = self._lib.kca_chan_recv(self._h, self.reader, self._buf, self._cap,
                                        1000 if self.block else self.timeout_ms, ctypes.byref(last))
            if n == -2 and self.block:
                continue
            if n < 0:  # -4: the writer died without closing (a blocking reader must not spin forever)
                raise ChannelError(f"shm channel recv failed ({n}: "
                                   f"{ {-2: 'timeout', -3: 'closed', -4: 'writer died'}.get(n, 'bad args') })")
            parts.append(self._buf.raw[:n])
            if last.value:
                break
        return pickle.loads(b"".join(parts))

    def close(self):
        if self._h:
            self._lib.kca_chan_close(self._h)
            self._h = None


def open_channel(group=None, src: int = 0, prefer: str | None = None):
    """Collective over ``group``: a shared-memory ring when all ranks share the
    writer's host and the native runtime loads (``KCA_TP_CTRL=gloo`` forces the
    gloo transport), else a gloo broadcast channel."""
    prefer = prefer or os.environ.get("KCA_TP_CTRL", "shm")
    rank = dist.get_rank(group)
    world = dist.get_world_size(group)
    ok = prefer == "shm"
    if ok:
        try:
            from ..io import native
            native.load()
        except Exception:  # noqa: BLE001 -- fall back to gloo
            ok = False
    info = [None] * world
    dist.all_gather_object(info, (socket.gethostname(), ok), group=group)
    if not all(o for _, o in info) or len({h for h, _ in info}) != 1:
        return GlooChannel(group, src)
    name = [f"/kca_tp_{os.getpid()}_{uuid.uuid4().hex[:12]}" if rank == src else None]
    dist.broadcast_object_list(name, src=src, group=group)
    ranks = sorted(r for r in range(world) if r != src)
    if rank == src:
        ch = ShmChannel(name[0], -1, readers=len(ranks))
        dist.barrier(group=group)
    else:
        dist.barrier(group=group)
        ch = ShmChannel(name[0], ranks.index(rank))
    return ch


__all__ = ["ShmChannel", "GlooChannel", "ChannelError", "open_channel"]
