"""Custom all-reduce over xGMI peer memory (csrc/comm/xgmi_allreduce.hip).

On an 8-GPU xGMI mesh every GPU has a direct link to every peer, so one kernel
that reads the peers' buffers concurrently beats RCCL's ring for the
tensor-parallel all-reduces (BLOOM TP=8 decode: two per layer of B x 14336
bf16; TP prefill and NeoX TP training: MB-sized, C12):

* ``one-shot`` up to ``one_shot_max`` bytes: one sync round, each rank reads
  the whole message from every peer (latency-bound sizes);
* ``two-shot`` up to ``max_bytes``: reduce-scatter + all-gather through peer
  memory, 2(W-1)/W of the message per rank over the links;
* larger messages keep going to RCCL (SURVEY §5.8 algorithm-by-size table).

Setup exchanges hipIpc handles of each rank's uncached staging/signal buffers
through ``torch.distributed`` (any backend) and maps the peers' buffers.
``all_reduce_(t)`` reduces a bf16 tensor in place and ``all_gather(t)``
concatenates every rank's ``t`` (the vocab-parallel LM head's logits); both are
graph-capturable (the call sequence number lives on the device), so a TP decode
graph holds no RCCL call at all. A peer that never arrives makes
the kernel time out: it poisons the output with NaN and sets a sticky error
word; ``check()`` raises on it (the TP engine calls it once per request).
"""
from __future__ import annotations

import ctypes
import os

import torch
import torch.distributed as dist

from ..ops import _lib

_REGISTRY: dict = {}

P = ctypes.c_void_p

ONE_SHOT, TWO_SHOT, ALL_GATHER = 0, 1, 2


def _fn(name, argtypes):
    lib = _lib.require()
    f = getattr(lib, name)
    f.argtypes = argtypes
    f.restype = ctypes.c_int
    return f


def pick(nbytes: int, world: int, one_shot_max: int) -> int:
    """Algorithm for a message of ``nbytes``: one-shot reads (W-1)*n bytes per
    rank in one round trip, two-shot 2(W-1)/W*n in two -- one-shot wins while
    the link latency dominates."""
    if world <= 2:
        return ONE_SHOT if nbytes <= 2 * one_shot_max else TWO_SHOT
    return ONE_SHOT if nbytes <= one_shot_max else TWO_SHOT


def blocks_for(n: int, world: int, algo: int, max_blocks: int = 128) -> int:
    """Workgroups: ~one 512-lane pass of 16-byte chunks per block per
    partition (two-shot) or of the whole message (one-shot)."""
    n8 = -(-n // 8)
    work = n8 if algo == ONE_SHOT else -(-n8 // world)
    return max(1, min(max_blocks, -(-work // 512)))


class AllReduceError(RuntimeError):
    pass


class XGMIAllReduce:
    def __init__(self, group=None, max_bytes: int = 64 << 20, one_shot_max: int = 256 << 10,
                 spin_limit: int = 1 << 26, local: bool = False):
        """``local=True``: a world-1 instance with no process group (parallel/tp_emulation.py: one rank of
        a TP layout on one GPU runs the deployment's all-reduce kernels -- staging, sync round, fused
        tails -- with itself as the only peer)."""
        self.group = group
        self.rank = 0 if local else dist.get_rank(group)
        self.world = 1 if local else dist.get_world_size(group)
        if self.world > 8:
            raise ValueError("xGMI all-reduce supports up to 8 ranks (one node)")
        self.max_bytes = max_bytes
        self.one_shot_max = one_shot_max
        self.spin_limit = spin_limit
        self.debug_delay = 0  # tests: spin before the read phase to force rank skew
        alloc = _fn("kca_ar_alloc", [ctypes.c_longlong, ctypes.POINTER(P)])
        ctl_alloc = _fn("kca_ar_ctl_alloc", [ctypes.POINTER(P)])
        handle = _fn("kca_ipc_handle", [P, P])
        self._open = _fn("kca_ipc_open", [P, ctypes.POINTER(P)])
        self._close = _fn("kca_ipc_close", [P])
        self._free = _fn("kca_ar_free", [P])
        run_args = [ctypes.POINTER(P), ctypes.POINTER(P), ctypes.POINTER(P), P, ctypes.c_int, ctypes.c_int,
                    ctypes.c_int, P, P, ctypes.c_longlong, ctypes.c_int, ctypes.c_longlong, ctypes.c_int, P]
        # element type -> entry (fp16: the serving precision of FT / DS-Inference; the kernels sum in fp32)
        self._runs = {torch.bfloat16: _fn("kca_ar_run", run_args), torch.float16: _fn("kca_ar_run_f16", run_args)}
        self._err = _fn("kca_ar_error", [P, ctypes.POINTER(ctypes.c_int)])
        ln_args = [ctypes.POINTER(P), ctypes.POINTER(P), ctypes.POINTER(P), P, ctypes.c_int, ctypes.c_int, P,
                   ctypes.c_int, ctypes.c_int, ctypes.c_longlong, P, P, P, P, P, ctypes.c_float, P, P, P, P, P, P, P]
        self._res_lns = {torch.bfloat16: _fn("kca_ar_res_ln", ln_args),
                         torch.float16: _fn("kca_ar_res_ln_f16", ln_args)}
        st_args = [ctypes.POINTER(P), ctypes.POINTER(P), ctypes.POINTER(P), P, ctypes.c_int, ctypes.c_int, P,
                   ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_longlong, P, P, P, ctypes.c_float, P, P, P, P]
        self._res_statss = {torch.bfloat16: _fn("kca_ar_res_stats", st_args),
                            torch.float16: _fn("kca_ar_res_stats_f16", st_args)}
        self._tails: dict = {}
        # batch-1 close: 0 = LayerNorm distributed over the launch (default), 1 = last-arriver tail (A/B)
        _fn("kca_ar_set_variant", [ctypes.c_int])(int(os.environ.get("KCA_AR_LN_VARIANT", "0")))
        self.res_ln_calls = 0  # fused tail launches (tests assert the TP decode layer took them)
        self.res_stats_calls = 0
        lib = _lib.require()
        self.max_blocks = int(lib.kca_ar_max_blocks())
        sig_bytes = lib.kca_ar_signal_bytes()
        own = []
        for nbytes in (max_bytes, max_bytes, sig_bytes):
            p = P()
            if alloc(nbytes, ctypes.byref(p)) != 0:
                raise RuntimeError("kca_ar_alloc failed")
            own.append(p.value)
        c = P()
        if ctl_alloc(ctypes.byref(c)) != 0:
            raise RuntimeError("kca_ar_ctl_alloc failed")
        self._ctl = c.value
        self._own = own
        hs = []
        for p in own:
            buf = ctypes.create_string_buffer(64)
            if handle(P(p), buf) != 0:
                raise RuntimeError("hipIpcGetMemHandle failed (is HSA_ENABLE_IPC_MODE_LEGACY=0 exported?)")
            hs.append(buf.raw)
        allh = [None] * self.world
        if local:
            allh[0] = hs
        else:
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
        self.calls = 0  # launches so far (tests check the xGMI path really carried the traffic)
        self._stage0 = arr(*ptrs[0])
        self._stage1 = arr(*ptrs[1])
        self._sig = arr(*ptrs[2])
        if not local:
            dist.barrier(group=group)

    def eligible(self, t: torch.Tensor) -> bool:
        return (t.is_cuda and t.dtype in (torch.bfloat16, torch.float16) and t.is_contiguous() and t.numel() % 8 == 0
                and 0 < t.numel() * 2 <= self.max_bytes and t.data_ptr() % 16 == 0)

    def all_reduce_(self, t: torch.Tensor, algo: int | None = None) -> torch.Tensor:
        n = t.numel()
        if not self.eligible(t):
            raise ValueError("tensor not eligible for the xGMI all-reduce (bf16/fp16, contiguous, 16B-aligned, "
                             f"numel % 8 == 0, <= {self.max_bytes} bytes)")
        if algo is None:
            algo = pick(2 * n, self.world, self.one_shot_max)
        blocks = blocks_for(n, self.world, algo, self.max_blocks)
        rc = self._runs[t.dtype](self._stage0, self._stage1, self._sig, P(self._ctl), self.rank, self.world, algo,
                       t.data_ptr(), t.data_ptr(), n, blocks, self.spin_limit, int(self.debug_delay),
                       _lib.stream())
        if rc != 0:
            raise RuntimeError(f"kca_ar_run status {rc}")
        self.calls += 1
        _lib.LAUNCHES[0] += 1
        return t

    def all_gather(self, t: torch.Tensor, out: torch.Tensor | None = None) -> torch.Tensor:
        """[world * t.numel()] bf16: rank r's ``t`` at ``out[r*n:(r+1)*n]``."""
        n = t.numel()
        if not self.eligible(t):
            raise ValueError("tensor not eligible for the xGMI all-gather (bf16/fp16, contiguous, 16B-aligned, "
                             f"numel % 8 == 0, <= {self.max_bytes} bytes)")
        if out is None:
            out = torch.empty(self.world * n, device=t.device, dtype=t.dtype)
        if out.numel() != self.world * n or not out.is_contiguous() or out.data_ptr() % 16:
            raise ValueError("all-gather output must be a contiguous 16B-aligned [world * n] tensor")
        blocks = blocks_for(n, self.world, ONE_SHOT, self.max_blocks)
        rc = self._runs[t.dtype](self._stage0, self._stage1, self._sig, P(self._ctl), self.rank, self.world, ALL_GATHER,
                       t.data_ptr(), out.data_ptr(), n, blocks, self.spin_limit, int(self.debug_delay),
                       _lib.stream())
        if rc != 0:
            raise RuntimeError(f"kca_ar_run (all-gather) status {rc}")
        self.calls += 1
        _lib.LAUNCHES[0] += 1
        return out

    def res_ln(self, t: torch.Tensor, bias, h: torch.Tensor, h_out: torch.Tensor, gamma: torch.Tensor, beta,
               eps: float, xn_out: torch.Tensor, gamma2=None, beta2=None, xn2_out=None) -> None:
        """Close a row-parallel projection of the batch-1 decode layer in ONE launch: all-reduce this
        rank's partial ``t`` ([1, N] bf16 or fp16), then h_out = bf16(h + sum + bias) and xn_out = LayerNorm(h_out)
        (and xn2_out with gamma2 / beta2) -- no bias add, no LayerNorm launch after the collective
        (``kca_ar_res_ln``; graph-capturable like ``all_reduce_``)."""
        n = t.numel()
        if not self.eligible(t) or n > 16384:
            raise ValueError("tensor not eligible for the fused all-reduce + LayerNorm (bf16/fp16 [N], N <= 16384)")
        ws = self._tail_ws(t.device)
        blocks = max(1, min(64, -(-(n // 8) // 128)))
        rc = self._res_lns[t.dtype](self._stage0, self._stage1, self._sig, P(self._ctl), self.rank, self.world, t.data_ptr(),
                          n, blocks, self.spin_limit, _lib.ptr(bias), h.data_ptr(), h_out.data_ptr(),
                          gamma.data_ptr(), _lib.ptr(beta), float(eps), xn_out.data_ptr(), _lib.ptr(gamma2),
                          _lib.ptr(beta2), _lib.ptr(xn2_out), ws[0].data_ptr(), ws[1].data_ptr(), _lib.stream())
        if rc != 0:
            raise RuntimeError(f"kca_ar_res_ln status {rc}")
        self.calls += 1
        self.res_ln_calls += 1
        _lib.LAUNCHES[0] += 1

    def res_stats(self, t: torch.Tensor, bias, h: torch.Tensor, h_out: torch.Tensor, stats, eps: float) -> None:
        """Close a row-parallel projection of the batch 2..64 matrix-core decode layer in ONE launch:
        all-reduce this rank's partial ``t`` ([M, N] bf16 or fp16), h_out = bf16(h + sum + bias), and the next
        LayerNorm's per-row (mean, rstd) into ``stats`` (an ``ops.skinny_mm.RowStatsBuf``), which the
        next projection applies on load (``kca_ar_res_stats``; graph-capturable)."""
        M, N = t.shape
        if not self.eligible(t) or N % 64 or N > 16384 or M > 64 or not h.is_contiguous() or h.shape != t.shape:
            raise ValueError("tensor not eligible for the fused all-reduce + row statistics (bf16 [M<=64, N], "
                             "N % 64 == 0, N <= 16384)")
        groups = t.numel() // 64
        blocks = max(1, min(self.max_blocks, -(-groups // 32)))
        from ..ops import skinny_mm as smm
        pub = smm.STATS_CONSUMER  # publish-only: 64-column slices, merged by the consuming projection
        rc = self._res_statss[t.dtype](self._stage0, self._stage1, self._sig, P(self._ctl), self.rank, self.world,
                             t.data_ptr(), M, N, blocks, self.spin_limit, _lib.ptr(bias), h.data_ptr(),
                             h_out.data_ptr(), float(eps), stats.part.data_ptr(),
                             None if pub else stats.stats.data_ptr(), stats.cnt.data_ptr(), _lib.stream())
        stats.nt, stats.eps = (N // 64 if pub else 0), float(eps)
        if rc != 0:
            raise RuntimeError(f"kca_ar_res_stats status {rc}")
        self.calls += 1
        self.res_stats_calls += 1
        _lib.LAUNCHES[0] += 1

    def _tail_ws(self, dev):
        """fp32 [16384] sums + the tail's zero-initialised arrival counters (local, not IPC-shared)."""
        ws = self._tails.get(str(dev))
        if ws is None:
            ws = (torch.zeros(16384, device=dev, dtype=torch.float32),  # (zeroed: tagged slots, see kernel)
                  torch.zeros(32 * 65, device=dev, dtype=torch.int32))
            self._tails[str(dev)] = ws
        return ws

    def error(self) -> int:
        e = ctypes.c_int(0)
        self._err(P(self._ctl), ctypes.byref(e))
        return e.value

    def check(self):
        """Raise if any call since setup timed out waiting for a peer (its
        output was NaN-poisoned). Synchronises the device."""
        e = self.error()
        if e:
            raise AllReduceError(f"xGMI all-reduce: peer did not arrive within the spin limit (error={e}); "
                                 "outputs of the affected calls are NaN")

    def close(self):
        for p in self._opened:
            self._close(P(p))
        for p in self._own:
            self._free(P(p))
        if self._ctl:
            self._free(P(self._ctl))
        self._opened, self._own, self._ctl = [], [], 0


def register(group=None, max_bytes: int = 64 << 20) -> XGMIAllReduce | None:
    """Enable the custom all-reduce for ``group`` (no-op off GPU or if disabled
    with KCA_CUSTOM_AR=0). An emulated TP group (parallel/tp_emulation.py) gets a rank-local
    instance, so the emulated rank runs the same tail kernels as a real rank."""
    if not torch.cuda.is_available() or os.environ.get("KCA_CUSTOM_AR", "1") == "0":
        return None
    from .tp_emulation import is_emulated
    if is_emulated(group):
        ar = XGMIAllReduce(None, max_bytes, local=True)
        _REGISTRY[id(group)] = ar
        return ar
    if dist.get_world_size(group) < 2:  # nothing to exchange
        return None
    ar = XGMIAllReduce(group, max_bytes)
    _REGISTRY[id(group)] = ar
    return ar


def lookup(group):
    return _REGISTRY.get(id(group))


def check_all():
    """Raise if any registered all-reduce timed out (call per request)."""
    for ar in _REGISTRY.values():
        ar.check()


__all__ = ["XGMIAllReduce", "AllReduceError", "register", "lookup", "check_all", "pick", "blocks_for"]
