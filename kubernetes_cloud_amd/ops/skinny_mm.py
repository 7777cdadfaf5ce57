"""Batched-decode GEMMs on the matrix cores (``csrc/kernels/skinny_mfma.hip``).

``y[M, N] = epilogue(x[M, K] . W[N, K]^T)`` for M = 2..64 decode rows (FasterTransformer's decoder at
batch > 1): the weight streams once from HBM straight into MFMA fragments, the activation rows are
re-read from L2, and the epilogues / prologues of a decode layer are folded in:

* ``act``: bias + GELU (fc_in);
* ``res``: bias + residual -> the new residual stream, with a **row-stats tail** (``stats=RowStatsBuf``)
  whose last-arriving workgroup writes the next LayerNorm's per-row (mean, rstd);
* ``ln=(stats, gamma, beta)`` on an input part: the activation is the residual stream, normalised on
  load with those statistics (no LayerNorm launch, no normalised-row buffer);
* two jobs per launch (N-concatenated, e.g. QKV and fc_in of a parallel-residual layer) or two
  K-concatenated parts of one job (GPT-J's ``o.Wo^T + g.Wf^T`` into one residual).

bf16 and fp16 (the precision FT / DS-Inference serve, BASELINE config 4). The descriptor is a
``ctypes.Structure`` mirroring ``MmArgs``; the entry point copies it into the kernel arguments, so a
launch is graph-capturable like any other.
"""
from __future__ import annotations

import ctypes
import os

import torch
import torch.nn.functional as F

from . import _lib

_P = ctypes.c_void_p
_LL = ctypes.c_longlong
_I = ctypes.c_int
_F = ctypes.c_float


class _Part(ctypes.Structure):
    _fields_ = [("x", _P), ("ldx", _LL), ("w", _P), ("ldw", _LL), ("K", _I), ("packed", _I), ("stats", _P),
                ("gamma", _P), ("beta", _P), ("st_nt", _I), ("st_eps", _F)]


class _Job(ctypes.Structure):
    _fields_ = [("p", _Part * 2), ("nparts", _I), ("N", _I), ("tiles", _I), ("bias", _P), ("act", _I), ("y", _P),
                ("ldy", _LL), ("res", _P), ("ldr", _LL), ("part", _P), ("stats_out", _P), ("cnt", _P),
                ("eps", _F)]


class _Args(ctypes.Structure):
    _fields_ = [("j", _Job * 2), ("njobs", _I), ("M", _I), ("ks", _I), ("nr", _I), ("kc", _I), ("wv", _I),
                ("ws", _P), ("bcnt", _P), ("ws_floats", _LL), ("bcnt_n", _I), ("pf", _I)]


_DT = {torch.bfloat16: 0, torch.float16: 1}
MAX_M = 64
# launch-shape knobs for same-box A/B runs (0 = the entry point's choice): K split over workgroups,
# 16-row weight tiles per wave
_KS = int(os.environ.get("KCA_MM_KS", "0"))
_NR = int(os.environ.get("KCA_MM_NR", "1"))
_KC = int(os.environ.get("KCA_MM_KC", "0"))  # K per chunk 128 / 256
_WV = int(os.environ.get("KCA_MM_WV", "0"))  # waves per workgroup 4 / 8
# split-K workspaces (fp32 partial tiles + zeroed per-block arrival counters), one per (device, stream):
# launches on one stream are ordered, launches on two streams must not share the counters
_WS: dict = {}
_ABI_OK = None


def _abi_ok() -> bool:
    global _ABI_OK
    if _ABI_OK is None:
        tgt = int(os.environ.get("KCA_MM_TARGET_WG", "0"))  # workgroups a K-split launch aims for (A/B)
        if tgt > 0:
            _lib.call("kca_mm_skinny_set", tgt)
        sizes = (ctypes.c_int * 3)()
        fn = getattr(_lib.require(), "kca_mm_skinny_abi")
        fn.argtypes = [ctypes.c_void_p]
        fn(ctypes.cast(sizes, ctypes.c_void_p))
        _ABI_OK = (sizes[0], sizes[1], sizes[2]) == (ctypes.sizeof(_Part), ctypes.sizeof(_Job), ctypes.sizeof(_Args))
        if not _ABI_OK:
            raise RuntimeError(f"kca_mm_skinny descriptor ABI mismatch: C {tuple(sizes)} vs ctypes "
                               f"{(ctypes.sizeof(_Part), ctypes.sizeof(_Job), ctypes.sizeof(_Args))}")
    return _ABI_OK


# consumer-side merge: the residual tails only publish per-slice (mean, M2) partials and the next
# projection merges them in its prologue (MmPart.st_nt) -- no arrival count / last-arriver merge on the
# producer. Same box, B=8: BLOOM rank 12.14 -> 11.92 ms, GPT-J 3.27 -> 3.21, NeoX 8.67 -> 8.71
# (profiles/mm_stats_consumer_ab_r6.jsonl); KCA_MM_STATS_CONSUMER=0: the producer merges (last arriver)
STATS_CONSUMER = os.environ.get("KCA_MM_STATS_CONSUMER", "1") not in ("0", "false")


class RowStatsBuf:
    """Workspace of one row-stats tail: per-tile partials, the (mean, rstd) output, arrival counters
    (zero-initialised, re-armed by every launch). One instance serves consecutive tails on a stream.
    ``nt`` > 0: the last producer left unmerged partials (``nt`` slices per row, ``eps`` for the
    consumer's merge) instead of merged stats (STATS_CONSUMER)."""

    def __init__(self, M: int, N: int, device):
        self.M, self.N = M, N
        self.part = torch.empty(M * (N // 16) * 2, device=device, dtype=torch.float32)
        self.stats = torch.zeros(M, 2, device=device, dtype=torch.float32)
        self.cnt = torch.zeros(32 * 65, device=device, dtype=torch.int32)
        self.nt, self.eps = 0, 1e-5

    def merged(self, M: int | None = None) -> torch.Tensor:
        """[M, 2] (mean, rstd) for host-side consumers: the kernel's merged stats, or the published
        partials merged here (the consumer kernels' equal-count Chan merge) when only those exist."""
        M = self.M if M is None else M
        if self.nt == 0:
            return self.stats[:M]
        p = self.part[:M * self.nt * 2].view(M, self.nt, 2)
        mt, qt = p[..., 0], p[..., 1]
        mean = mt.mean(1, keepdim=True)
        m2 = qt.sum(1, keepdim=True) + (self.N / self.nt) * ((mt - mean) ** 2).sum(1, keepdim=True)
        return torch.cat([mean, torch.rsqrt(m2 / self.N + self.eps)], dim=1)


def supported(x: torch.Tensor, w: torch.Tensor) -> bool:
    """Shapes / dtypes the MFMA kernel takes (the caller falls back otherwise)."""
    M, K = x.shape
    return (x.is_cuda and x.dtype in _DT and w.dtype == x.dtype and 1 <= M <= MAX_M and K % 8 == 0
            and x.stride(1) == 1 and x.stride(0) % 8 == 0 and w.stride(1) == 1 and w.stride(0) % 8 == 0
            and x.data_ptr() % 16 == 0 and w.data_ptr() % 16 == 0 and w.shape[1] == K)


# packed weight stream (pack_weight): the decode runner keeps a packed twin of every weight the batched
# layer streams (KCA_MM_PACK=0: the row-major weights themselves)
PACK = os.environ.get("KCA_MM_PACK", "1") not in ("0", "false")


def pack_weight(w: torch.Tensor) -> torch.Tensor:
    """[N, K] -> the kernel's packed stream layout [ceil(N/16), ceil(K/128), 16, 128], zero-padded: each
    wave's 16-row x 128-column sub-tile is one contiguous 4 KB block (``MmPart.packed``)."""
    N, K = w.shape
    Np, Kp = -(-N // 16) * 16, -(-K // 128) * 128
    if (Np, Kp) != (N, K):
        wz = w.new_zeros(Np, Kp)
        wz[:N, :K] = w
        w = wz
    return w.reshape(Np // 16, 16, Kp // 128, 128).permute(0, 2, 1, 3).contiguous()


def part(x, w, ln=None, packed=None):
    """One K-part: x [M, K], w [N, K]; ``ln=(stats [M, 2] fp32, gamma, beta)`` normalises x on load;
    ``packed``: ``pack_weight(w)``, streamed instead of w."""
    p = _Part()
    p.x, p.ldx, p.w, p.ldw, p.K = x.data_ptr(), x.stride(0), w.data_ptr(), w.stride(0), x.shape[1]
    if packed is not None:
        p.w, p.ldw, p.packed = packed.data_ptr(), packed.shape[1] * 16 * 128, 1
    if ln is not None:
        st, g, b = ln
        if isinstance(st, RowStatsBuf):
            if st.nt > 0:  # unmerged partials: the kernel merges them (MmPart.st_nt)
                p.stats, p.st_nt, p.st_eps = st.part.data_ptr(), st.nt, st.eps
            else:
                p.stats = st.stats.data_ptr()
        else:
            p.stats = st.data_ptr()
        p.gamma, p.beta = g.data_ptr(), _lib.ptr(b)
    return p


def job(parts, N: int, y: torch.Tensor, bias=None, act: int = 0, res=None, stats: RowStatsBuf | None = None,
        eps: float = 1e-5):
    j = _Job()
    for i, p in enumerate(parts):
        j.p[i] = p
    j.nparts, j.N, j.bias, j.act = len(parts), N, _lib.ptr(bias), int(act)
    j.y, j.ldy = y.data_ptr(), y.stride(0)
    if res is not None:
        j.res, j.ldr = res.data_ptr(), res.stride(0)
    if stats is not None:
        if STATS_CONSUMER:  # publish-only tail: 16-column slices, merged by the consumer
            j.part, j.eps = stats.part.data_ptr(), eps
            stats.nt, stats.eps = N // 16, eps
        else:
            j.part, j.stats_out, j.cnt, j.eps = stats.part.data_ptr(), stats.stats.data_ptr(), stats.cnt.data_ptr(), eps
            stats.nt = 0
    return j


def _workspace(device, floats: int, nblk: int):
    key = (str(device), torch.cuda.current_stream(device).cuda_stream)
    ws = _WS.get(key)
    if ws is None or ws[0].numel() < floats or ws[1].numel() < nblk:
        f = max(floats, ws[0].numel() if ws else 0, 1 << 20)
        n = max(nblk, ws[1].numel() if ws else 0, 4096)
        ws = (torch.empty(f, device=device, dtype=torch.float32), torch.zeros(n, device=device, dtype=torch.int32))
        _WS[key] = ws
    return ws


def plan(jobs, M: int, dtype: torch.dtype, ks: int | None = None, nr: int | None = None):
    """(K split, workspace floats, block counters) the entry point picks for these jobs."""
    a = _args(jobs, M, ks, nr)
    wsf, nb, k = ctypes.c_longlong(0), ctypes.c_int(0), ctypes.c_int(0)
    fn = _lib.require().kca_mm_skinny_plan
    fn.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]
    fn.restype = ctypes.c_int
    rc = fn(ctypes.addressof(a), _DT[dtype], ctypes.addressof(wsf), ctypes.addressof(nb), ctypes.addressof(k))
    if rc != 0:
        raise RuntimeError(f"kca_mm_skinny_plan returned status {rc} (unsupported shape/arguments)")
    return k.value, wsf.value, nb.value


def _args(jobs, M, ks, nr):
    _abi_ok()
    a = _Args()
    for i, j in enumerate(jobs):
        a.j[i] = j
    a.njobs, a.M = len(jobs), M
    a.ks = _KS if ks is None else ks
    a.nr = _NR if nr is None else nr
    a.kc, a.wv = _KC, _WV
    return a


def launch(jobs, M: int, dtype: torch.dtype, ks: int | None = None, nr: int | None = None) -> None:
    """One kernel launch over 1-2 jobs on the current stream."""
    k, wsf, nb = plan(jobs, M, dtype, ks, nr)
    a = _args(jobs, M, ks, nr)
    if k > 1:
        dev = torch.device("cuda", torch.cuda.current_device())
        ws, bc = _workspace(dev, wsf, nb)
        a.ws, a.bcnt, a.ws_floats, a.bcnt_n = ws.data_ptr(), bc.data_ptr(), ws.numel(), bc.numel()
    fn = _lib.require().kca_mm_skinny
    fn.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p]
    fn.restype = ctypes.c_int
    rc = fn(ctypes.addressof(a), _DT[dtype], _lib.stream())
    if rc != 0:
        raise RuntimeError(f"kca_mm_skinny returned status {rc} (unsupported shape/arguments)")
    _lib.LAUNCHES[0] += 1
    if _lib.SYNC_LAUNCH:
        torch.cuda.synchronize()


def mm(x: torch.Tensor, w: torch.Tensor, bias=None, act: int = 0, out=None, res=None, stats=None, eps=1e-5,
       ln=None, packed=None) -> torch.Tensor:
    """Single-job convenience: ``act(LN?(x) W^T + b) (+ res)``."""
    M = x.shape[0]
    N = w.shape[0]
    if out is None:
        out = torch.empty(M, N, device=x.device, dtype=x.dtype)
    launch([job([part(x, w, ln, packed)], N, out, bias, act, res, stats, eps)], M, x.dtype)
    return out


# ----------------------------------------------------------------------------- reference math (fp32)
def _act_ref(y, act):
    if act == 1:
        return F.gelu(y, approximate="tanh")
    if act == 2:
        return F.gelu(y)
    return y


def ln_on_load_reference(h, stats, gamma, beta):
    """The prologue: (h - mean) * rstd * gamma + beta, rounded to h's dtype."""
    hf = h.float()
    y = (hf - stats[:, :1]) * stats[:, 1:] * gamma.float() + (0 if beta is None else beta.float())
    return y.to(h.dtype)


def row_stats_reference(h, eps):
    """(mean, rstd) per row of the rounded residual stream (fp32, two-pass)."""
    hf = h.float()
    mean = hf.mean(-1, keepdim=True)
    var = ((hf - mean) ** 2).mean(-1, keepdim=True)
    return torch.cat([mean, torch.rsqrt(var + eps)], dim=1)


def mm_reference(parts, bias=None, act=0, res=None, dtype=torch.bfloat16):
    """parts: [(x, w, ln)] -> the job's output (rounded to dtype) in fp32 math."""
    y = None
    for x, w, ln in parts:
        xx = x if ln is None else ln_on_load_reference(x, *ln)
        t = xx.float() @ w.float().t()
        y = t if y is None else y + t
    if bias is not None:
        y = y + bias.float()
    y = _act_ref(y, act)
    if res is not None:
        y = y + res.float()
    return y.to(dtype)


__all__ = ["RowStatsBuf", "supported", "part", "job", "launch", "mm", "mm_reference", "row_stats_reference",
           "ln_on_load_reference", "MAX_M"]
