"""ctypes binding of the in-tree gfx950 kernel library (``_lib/libkca_kernels.so``).

The library is a plain C-ABI shared object built by ``tools/build_ext.py``
(``hipcc --offload-arch=gfx950``). It is loaded *after* ``import torch`` so the
kernels register with the HIP runtime torch already mapped; every launch takes
the current torch stream, so launches are ordered with torch's own work and
are captured by ``torch.cuda.graphs`` like any other kernel.

Policy: GPU tensors always go through the native kernels. If the library is
missing on a machine with a GPU the ops raise (``require()``) instead of
silently falling back to eager PyTorch -- CPU tensors use the reference
implementations in each op module (that is what the CPU test-suite runs).
"""
from __future__ import annotations

import ctypes
import os
import threading

import torch

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_DIR = os.path.join(os.path.dirname(_HERE), "_lib")
# KCA_DEBUG=1: the debug build (KCA_DASSERT bounds/invariant checks in the kernels)
DEBUG = os.environ.get("KCA_DEBUG", "0") in ("1", "true")
KERNEL_LIB = os.path.join(LIB_DIR, "libkca_kernels_debug.so" if DEBUG else "libkca_kernels.so")
# KCA_KERNEL_LIB=<path>: load another build of the kernel library (same-box A/B of a kernel change)
KERNEL_LIB = os.environ.get("KCA_KERNEL_LIB") or KERNEL_LIB

_lock = threading.Lock()
_lib = None
_err: str | None = None

P = ctypes.c_void_p
I = ctypes.c_int
LL = ctypes.c_longlong
F = ctypes.c_float

# name -> argtypes (restype is always int status, 0 == ok)
_SIGS = {
    "kca_layernorm_fwd": [P, P, P, P, P, P, P, P, P, I, I, F, P],
    "kca_gemm_lt": [P, LL, P, LL, P, P, LL, P, LL, I, I, I, F, P, LL, P],
    "kca_gemm_lt_gelu": [P, LL, P, LL, I, P, P, LL, P, LL, I, I, I, P, LL, P],
    "kca_layernorm_bwd_parts": [I],
    "kca_layernorm_bwd": [P, P, P, P, P, P, P, P, P, I, P, I, I, P],
    "kca_gelu_fwd": [P, P, LL, I, P],
    "kca_gelu_fwd_f16": [P, P, LL, I, P],
    "kca_gelu_bwd": [P, P, P, LL, I, P],
    "kca_quick_gelu_fwd": [P, P, LL, P],
    "kca_quick_gelu_bwd": [P, P, P, LL, P],
    "kca_geglu_fwd": [P, P, LL, I, P],
    "kca_add_bias_nhwc": [P, P, P, P, LL, I, P],
    "kca_add_bias2_nhwc": [P, P, P, P, P, LL, I, P],
    "kca_colsum_bf16": [P, P, I, I, I, P],
    "kca_geglu_bwd": [P, P, P, LL, I, P],
    "kca_rope": [P, P, I, I, LL, I, LL, LL, LL, LL, I, I, P, P, P, F, P],
    "kca_accum_grad": [P, P, F, I, LL, P],
    "kca_accum_grad_pair": [P, P, P, F, LL, P],
    "kca_accum_grad_multi": [P, I, F, P],
    "kca_cast_f32_bf16": [P, P, LL, P],
    "kca_ema": [P, P, F, LL, P],
    "kca_cross_entropy_fwd": [P, LL, P, I, I, I, P, P, P],
    "kca_cross_entropy_bwd": [P, LL, P, P, P, F, I, I, I, P, LL, P],
    "kca_adamw": [P, P, P, P, P, LL, P, F, F, F, F, F, F, F, P, P, P],
    "kca_sumsq": [P, LL, P, P, P],
    "kca_adamw8bit": [P, P, P, P, P, P, P, LL, P, F, F, F, F, F, F, F, P, P, P],
    "kca_clip_coef": [P, F, F, P, P, P, P],
    "kca_attn_fwd": [P] * 5 + [LL] * 12 + [I] * 7 + [F, P, P, I, P, I, I, P, P],
    "kca_attn_bwd_preprocess": [P, P, P, LL, LL, LL, LL, LL, LL, I, I, I, I, P],
    "kca_attn_bwd": [P] * 10 + [LL] * 21 + [I] * 7 + [F, P, P, I, P, P],
    "kca_attn_fwd_wide": [P] * 5 + [LL] * 12 + [I] * 6 + [F, P, P],
    "kca_attn_set_tiled": [I],
    "kca_attn_set_variant": [I],
    "kca_transpose_bf16": [P, LL, P, LL, I, I, P],
    "kca_gelu_fwd_t": [P, LL, P, LL, P, LL, I, I, I, P],
    "kca_gelu_bwd_t": [P, LL, P, LL, P, LL, P, LL, P, I, I, I, P],
    "kca_transpose_colsum": [P, LL, P, LL, P, I, I, P],
    "kca_col_reduce_f32": [P, I, I, P, P, P],
    "kca_accum_grad_2d": [P, P, LL, I, I, F, I, P],
    "kca_groupnorm_fwd": [P, P, P, P, P, P, P, I, I, I, I, F, I, P],
    "kca_groupnorm_bwd": [P, P, P, P, P, P, P, P, P, P, I, I, I, I, I, P],
    "kca_groupnorm_nhwc_ws": [I, I, I],
    "kca_groupnorm_nhwc_fwd": [P, P, P, P, P, P, P, I, I, I, I, F, I, P],
    "kca_groupnorm_nhwc_fwd_add": [P, P, P, P, LL, P, P, P, P, I, I, I, I, F, I, P],
    "kca_groupnorm_nhwc_cat_fwd": [P, P, P, P, P, P, P, P, P, P, I, I, I, I, I, I, F, I, P],
    "kca_groupnorm_nhwc_bwd": [P, P, P, P, P, P, P, P, P, P, I, I, I, I, I, P],
    "kca_skinny_set_smallk": [I],
    "kca_conv3x3_fwd": [P, P, P, P, I, I, I, I, I, P],
    "kca_conv3x3_set_variant": [I],
    "kca_skinny_gemm": [P, LL, P, P, P, LL, I, I, I, I, P],
    "kca_skinny_set_splitk": [I],
    "kca_mm_skinny_set": [I],
    "kca_ln_skinny_gemm": [P, LL, P, P, P, LL, P, P, F, P, P, P, LL, I, I, I, I, P, P],
    "kca_ln_rows": [P, LL, P, P, P, LL, P, P, F, P, I, I, P],
    "kca_embed_ln_rows": [P, LL, P, P, P, I, P, LL, P, P, F, P, I, I, P],
    "kca_decode_prep": [P, LL, I, I, I, I, I, I, P, P, P, P, P, P, LL, LL, LL, P, I, I, P],
    "kca_decode_chunk": [I, I, I],
    "kca_decode_set_stamps": [P],
    "kca_decode_attn": [P, LL, P, P, LL, LL, LL, P, P, P, LL, P, LL, I, I, I, I, I, I, F, P, P, I, I, I, P],
    "kca_sd_noise_prep": [P, P, P, P, P, P, P, P, P, I, I, I, I, F, I, ctypes.c_ulonglong, LL, I, P],
    "kca_mse_split_fwd": [P, P, LL, LL, F, P, I, P, P],
    "kca_mse_split_bwd": [P, P, P, LL, LL, F, P, P],
    "kca_sd_lms_step": [P, P, P, P, LL, P, I, I, I, I, I, F, F, F, P],
    "kca_decode_prep_attn": [P, LL, P, P, LL, LL, LL, P, P, P, LL, P, LL, I, I, I, I, I, I, F, P, P, I, I, I, I, P,
                             P, I, I, P],
    "kca_im2col2x2_nhwc": [P, P, I, I, I, I, P],
    "kca_phase_to_dense_nhwc": [P, P, P, I, I, I, I, P],
    "kca_upsample2x_nhwc": [P, P, I, I, I, I, P],
    "kca_dense_to_phase_nhwc": [P, P, I, I, I, I, P],
    "kca_col2im2x2_nhwc": [P, P, I, I, I, I, P],
    "kca_pad_br_nhwc": [P, P, I, I, I, I, P],
    "kca_gemv_dual_ln": [P, P, I, P, P, I, P, P, P, P, P, P, P, F, P, P, P, P, I, P],
    "kca_sample_logits": [P, LL, I, I, I, P, P, P, P, P, P, P, I, P, LL, P, P, P, P, P, I, P],
}


# fused decode layer (batch 1): kca_decode_prep_attn's arguments (minus the stream), then the fc_in
# GEMV's x, W, bias, y, N, K, act, then the stream
_SIGS["kca_decode_prep_attn_gemv"] = _SIGS["kca_decode_prep_attn"][:-2] + [P, P, P, P, I, I, I, I, P]

# fp16 twins of the serving kernels (same arguments)
for _n in ("kca_decode_prep_attn", "kca_ln_rows", "kca_embed_ln_rows", "kca_decode_prep_attn_gemv",
           "kca_gemv_dual_ln", "kca_skinny_gemm"):
    _SIGS[_n + "_f16"] = _SIGS[_n]


def _load():
    global _lib, _err
    if _lib is not None or _err is not None:
        return _lib
    with _lock:
        if _lib is not None or _err is not None:
            return _lib
        if not os.path.exists(KERNEL_LIB):
            _err = f"{KERNEL_LIB} not built (run `python tools/build_ext.py`)"
            return None
        try:
            lib = ctypes.CDLL(KERNEL_LIB, mode=ctypes.RTLD_GLOBAL)
        except OSError as e:  # pragma: no cover - depends on the box
            _err = f"failed to load {KERNEL_LIB}: {e}"
            return None
        for name, argtypes in _SIGS.items():
            fn = getattr(lib, name, None)
            if fn is None:
                continue
            fn.argtypes = argtypes
            fn.restype = ctypes.c_int
        _lib = lib
        return _lib


def available() -> bool:
    return _load() is not None


def require():
    lib = _load()
    if lib is None:
        raise RuntimeError(
            "kubernetes_cloud_amd native kernels unavailable: " + str(_err)
            + " -- refusing to fall back to eager PyTorch on a GPU tensor")
    return lib


def has(name: str) -> bool:
    lib = _load()
    return lib is not None and hasattr(lib, name)


# KCA_SYNC_LAUNCH=1: synchronise after every native launch so an asynchronous
# GPU fault (out-of-bounds access, illegal instruction) is reported at the op
# that caused it, by name -- the HIP_LAUNCH_BLOCKING-style debug mode of
# SURVEY §5.2. Off by default (it serialises the stream).
SYNC_LAUNCH = os.environ.get("KCA_SYNC_LAUNCH", "0") in ("1", "true")


# native launches issued through this module, ops/skinny_mm.py and parallel/custom_ar.py (the serving
# runner reports launches per decode step from it)
LAUNCHES = [0]


def call(name: str, *args):
    lib = require()
    fn = getattr(lib, name)
    LAUNCHES[0] += 1
    rc = fn(*args)
    if rc != 0:
        raise RuntimeError(f"{name} returned status {rc} (unsupported shape/arguments)")
    if SYNC_LAUNCH and torch.cuda.is_available():
        try:
            torch.cuda.synchronize()
        except RuntimeError as e:  # pragma: no cover - needs a faulting kernel
            raise RuntimeError(f"GPU fault after native launch {name}: {e}") from e
    return rc


def call_rc(name: str, *args) -> int:
    """``call`` for entry points whose nonzero status means "shape outside this kernel" (the caller
    takes another path) rather than an error."""
    rc = getattr(require(), name)(*args)
    LAUNCHES[0] += rc == 0
    if rc == 0 and SYNC_LAUNCH and torch.cuda.is_available():
        torch.cuda.synchronize()
    return rc


def stream() -> int:
    return torch.cuda.current_stream().cuda_stream


def ptr(t: torch.Tensor | None) -> int | None:
    return None if t is None else t.data_ptr()


def native_f16(*tensors: torch.Tensor | None) -> bool:
    """True for fp16 GPU tensors (all of them): the serving kernels with fp16 twins
    (``*_f16`` entry points) take them natively -- the precision FasterTransformer and
    DS-Inference serve (BASELINE config 4)."""
    on_gpu = False
    for t in tensors:
        if t is not None and t.is_cuda:
            on_gpu = True
            if t.dtype != torch.float16:
                return False
    return on_gpu


def use_native(*tensors: torch.Tensor | None) -> bool:
    """True when the op must run on the native HIP path.

    Native kernels are bf16; a GPU tensor of another dtype (fp32 debugging runs)
    uses the reference math. bf16 GPU tensors never fall back: a missing
    library raises in ``call``.
    """
    on_gpu = False
    for t in tensors:
        if t is not None and t.is_cuda:
            on_gpu = True
            if t.dtype != torch.bfloat16:
                return False
    return on_gpu
