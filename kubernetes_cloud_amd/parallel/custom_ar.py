"""Custom one-shot all-reduce over xGMI peer memory (csrc/comm/xgmi_allreduce.hip).

For the latency-bound all-reduces of tensor-parallel decode (BLOOM TP=8: two
per layer, B x 14336 bf16 each) a single kernel that reads the 7 peers'
buffers directly over the point-to-point links beats RCCL's ring; larger
messages keep going to RCCL (SURVEY §5.8 algorithm-by-size table).

Setup exchanges hipIpc handles of each rank's uncached staging/signal buffers
through ``torch.distributed`` (any backend) and maps the peers' buffers.
``all_reduce_(t)`` reduces a bf16 tensor in place and is graph-capturable.
``register(group)`` makes ``tensor_parallel.reduce_from_tp`` use it for
messages up to ``max_bytes``.
"""
from __future__ import annotations

import ctypes
import os

import torch
import torch.distributed as dist

from ..ops import _lib

_REGISTRY: dict = {}

P = ctypes.c_void_p


def _fn(name, argtypes):
    lib = _lib.require()
    f = getattr(lib, name)
    f.argtypes = argtypes
    f.restype = ctypes.c_int
    return f


class XGMIAllReduce:
    def __init__(self, group=None, max_bytes: int = 4 << 20, spin_limit: int = 1 << 26):
        self.group = group
        self.rank = dist.get_rank(group)
        self.world = dist.get_world_size(group)
        if self.world > 8:
            raise ValueError("one-shot all-reduce supports up to 8 ranks (one node)")
        self.max_bytes = max_bytes
        self.spin_limit = spin_limit
        alloc = _fn("kca_ar_alloc", [ctypes.c_longlong, ctypes.POINTER(P)])
        handle = _fn("kca_ipc_handle", [P, P])
        self._open = _fn("kca_ipc_open", [P, ctypes.POINTER(P)])
        self._close = _fn("kca_ipc_close", [P])
        self._free = _fn("kca_ar_free", [P])
        self._run = _fn("kca_ar_one_shot", [ctypes.POINTER(P), ctypes.POINTER(P), ctypes.POINTER(P), ctypes.c_int,
                                            ctypes.c_int, P, P, ctypes.c_longlong, ctypes.c_int, ctypes.c_longlong,
                                            P])
        sig_bytes = _lib.require().kca_ar_signal_bytes()
        own = []
        for nbytes in (max_bytes, max_bytes, sig_bytes):
            p = P()
            if alloc(nbytes, ctypes.byref(p)) != 0:
                raise RuntimeError("kca_ar_alloc failed")
            own.append(p.value)
        self._own = own
        hs = []
        for p in own:
            buf = ctypes.create_string_buffer(64)
            if handle(P(p), buf) != 0:
                raise RuntimeError("hipIpcGetMemHandle failed (is HSA_ENABLE_IPC_MODE_LEGACY=0 exported?)")
            hs.append(buf.raw)
        allh = [None] * self.world
        dist.all_gather_object(allh, hs, group=group)
        self._opened = []
        ptrs = [[0] * self.world for _ in range(3)]
        for r in range(self.world):
            for i in range(3):
                if r == self.rank:
                    ptrs[i][r] = own[i]
                else:
                    q = P()
                    if self._open(ctypes.create_string_buffer(allh[r][i], 64), ctypes.byref(q)) != 0:
                        raise RuntimeError(f"hipIpcOpenMemHandle failed for rank {r}")
                    ptrs[i][r] = q.value
                    self._opened.append(q.value)
        arr = P * self.world
        self._stage0 = arr(*ptrs[0])
        self._stage1 = arr(*ptrs[1])
        self._sig = arr(*ptrs[2])
        self.sig_own = own[2]
        dist.barrier(group=group)

    def eligible(self, t: torch.Tensor) -> bool:
        return (t.is_cuda and t.dtype == torch.bfloat16 and t.is_contiguous() and t.numel() % 8 == 0
                and t.numel() * 2 <= self.max_bytes and t.data_ptr() % 16 == 0)

    def all_reduce_(self, t: torch.Tensor) -> torch.Tensor:
        n = t.numel()
        blocks = max(1, min(64, -(-n // (8 * 256))))
        rc = self._run(self._stage0, self._stage1, self._sig, self.rank, self.world, t.data_ptr(), t.data_ptr(),
                       n, blocks, self.spin_limit, _lib.stream())
        if rc != 0:
            raise RuntimeError(f"kca_ar_one_shot status {rc}")
        return t

    def error(self) -> int:
        f = _fn("kca_ar_error", [P, ctypes.POINTER(ctypes.c_int)])
        e = ctypes.c_int(0)
        f(P(self.sig_own), ctypes.byref(e))
        return e.value

    def close(self):
        for p in self._opened:
            self._close(P(p))
        for p in self._own:
            self._free(P(p))
        self._opened, self._own = [], []


def register(group=None, max_bytes: int = 4 << 20) -> XGMIAllReduce | None:
    """Enable the custom all-reduce for ``group`` (no-op off GPU or if disabled
    with KCA_CUSTOM_AR=0)."""
    if not torch.cuda.is_available() or os.environ.get("KCA_CUSTOM_AR", "1") == "0":
        return None
    ar = XGMIAllReduce(group, max_bytes)
    _REGISTRY[id(group)] = ar
    return ar


def lookup(group):
    return _REGISTRY.get(id(group))


__all__ = ["XGMIAllReduce", "register", "lookup"]
