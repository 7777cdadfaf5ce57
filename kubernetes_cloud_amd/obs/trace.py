"""Tracing hooks: roctx ranges, optional torch-profiler export.

``trace_range("fwd")`` pushes/pops a roctx range through the ROCm 7
``librocprofiler-sdk-roctx`` C API, so phases (forward, backward, optimizer,
comm, decode step) show up as named regions in ``rocprofv3 --marker-trace``
timelines around the kernels they launch. Without the library (CPU boxes) the
ranges are no-ops. ``KCA_ROCTX=0`` disables them.

``maybe_profile(dir)`` wraps a region in ``torch.profiler`` with a Chrome-trace
export when ``KCA_TORCH_PROFILE=1`` -- the reference only had W&B timings
(finetuner-workflow/finetuner/finetuner.py:496-535).
"""
from __future__ import annotations

import contextlib
import ctypes
import ctypes.util
import os

_roctx = None
_tried = False


def _lib():
    global _roctx, _tried
    if _tried:
        return _roctx
    _tried = True
    if os.environ.get("KCA_ROCTX", "1") in ("0", "false"):
        return None
    rocm = os.environ.get("ROCM_PATH", "/opt/rocm")
    for name in (os.path.join(rocm, "lib", "librocprofiler-sdk-roctx.so.1"),
                 os.path.join(rocm, "lib", "librocprofiler-sdk-roctx.so"),
                 ctypes.util.find_library("rocprofiler-sdk-roctx") or ""):
        if name and os.path.exists(name):
            try:
                lib = ctypes.CDLL(name)
                lib.roctxRangePushA.argtypes = [ctypes.c_char_p]
                lib.roctxRangePushA.restype = ctypes.c_int
                lib.roctxRangePop.restype = ctypes.c_int
                lib.roctxMarkA.argtypes = [ctypes.c_char_p]
                _roctx = lib
                break
            except (OSError, AttributeError):
                continue
    return _roctx


def available() -> bool:
    return _lib() is not None


@contextlib.contextmanager
def trace_range(name: str):
    lib = _lib()
    if lib is None:
        yield
        return
    lib.roctxRangePushA(name.encode())
    try:
        yield
    finally:
        lib.roctxRangePop()


def mark(name: str) -> None:
    lib = _lib()
    if lib is not None:
        lib.roctxMarkA(name.encode())


@contextlib.contextmanager
def maybe_profile(out_dir: str, name: str = "trace"):
    if os.environ.get("KCA_TORCH_PROFILE", "0") not in ("1", "true"):
        yield None
        return
    import torch

    acts = [torch.profiler.ProfilerActivity.CPU]
    if torch.cuda.is_available():
        acts.append(torch.profiler.ProfilerActivity.CUDA)
    os.makedirs(out_dir, exist_ok=True)
    with torch.profiler.profile(activities=acts, record_shapes=True) as prof:
        yield prof
    prof.export_chrome_trace(os.path.join(out_dir, f"{name}.json"))
