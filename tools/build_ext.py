#!/usr/bin/env python3
"""Build the native libraries of kubernetes_cloud_amd in-tree.

* ``libkca_kernels.so`` -- every ``csrc/kernels/*.hip`` compiled by ``hipcc
  --offload-arch=gfx950`` (CDNA4 only; no other targets, no hipify step).
* ``libkca_host.so``    -- host-side C++ runtime pieces (``csrc/cpu``,
  ``csrc/io``, ``csrc/tokenize``): AVX-512/AVX2 AdamW for offload, the
  ``.tensors`` weight streamer, the BPE tokenizer / context packer and the
  shared-memory control channel of the TP serving engine (``csrc/runtime``).

Both are plain C-ABI shared objects loaded with ctypes *after* ``import
torch`` so that the HIP runtime torch already mapped (soname
``libamdhip64.so.7``) is the one the kernels register with.

Objects are cached by content hash under ``build/`` so a rebuild after a
one-file edit only recompiles that file.
"""
from __future__ import annotations

import argparse
import concurrent.futures as cf
import hashlib
import os
import shutil
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "csrc")
OUT_DIR = os.path.join(ROOT, "kubernetes_cloud_amd", "_lib")
BUILD = os.path.join(ROOT, "build")
ROCM = os.environ.get("ROCM_PATH", "/opt/rocm")
HIPCC = os.path.join(ROCM, "bin", "hipcc")

ARCH = "gfx950"
HIP_FLAGS = [
    f"--offload-arch={ARCH}", "-O3", "-fPIC", "-std=c++17",
    "-munsafe-fp-atomics", "-Wno-unused-result", "-fvisibility=hidden",
]
HOST_FLAGS = ["-O3", "-fPIC", "-std=c++17", "-fopenmp", "-fvisibility=hidden",
              "-Wall", "-Wno-unused-function"]


def _hash(paths, flags):
    h = hashlib.sha1()
    for p in sorted(paths):
        with open(p, "rb") as f:
            h.update(f.read())
    h.update(" ".join(flags).encode())
    return h.hexdigest()[:16]


def _compile(cmd_base, src, deps, obj_dir, flags):
    key = _hash([src] + deps, flags)
    obj = os.path.join(obj_dir, os.path.basename(src) + f".{key}.o")
    if os.path.exists(obj):
        return obj
    cmd = cmd_base + flags + ["-c", src, "-o", obj + ".tmp"]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"compile failed: {' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
    os.replace(obj + ".tmp", obj)
    return obj


def _sources(sub, exts):
    d = os.path.join(CSRC, sub)
    if not os.path.isdir(d):
        return []
    return sorted(os.path.join(d, f) for f in os.listdir(d) if f.endswith(exts))


def build_kernels(jobs: int = 8, verbose: bool = False, debug: bool = False, stamps: bool = False,
                  ab_define: str | None = None) -> str:
    """``debug``: libkca_kernels_debug.so with the KCA_DASSERT bounds checks
    compiled in (csrc/kernels/common.h), loaded by ops/_lib.py when KCA_DEBUG=1.
    ``stamps``: ab/libkca_kernels_stamps.so, the diagnostic build with the
    attention kernels' in-loop s_memtime segment sums (bench/attn_stamps.py,
    loaded through KCA_KERNEL_LIB); never the library the framework loads.
    ``ab_define``: ab/libkca_kernels_<define>.so built with -D<define>, the
    other arm of a same-box A/B (loaded through KCA_KERNEL_LIB)."""
    srcs = _sources("kernels", (".hip",)) + _sources("comm", (".hip",))
    hdrs = _sources("kernels", (".h",)) + _sources("comm", (".h",))
    obj_dir = os.path.join(BUILD, "kernels_debug" if debug else ("kernels_stamps" if stamps else "kernels"))
    if ab_define:
        obj_dir = os.path.join(BUILD, "kernels_" + ab_define.lower())
    os.makedirs(obj_dir, exist_ok=True)
    os.makedirs(OUT_DIR, exist_ok=True)
    flags = HIP_FLAGS + (["-DKCA_DEBUG", "-g"] if debug else []) + (["-DKCA_ATTN_STAMPS"] if stamps else []) + (
        [f"-D{ab_define}"] if ab_define else [])
    with cf.ThreadPoolExecutor(max_workers=jobs) as ex:
        objs = list(ex.map(lambda s: _compile([HIPCC], s, hdrs, obj_dir, flags), srcs))
    out = os.path.join(OUT_DIR, "libkca_kernels_debug.so" if debug else "libkca_kernels.so")
    if stamps:
        os.makedirs(os.path.join(ROOT, "ab"), exist_ok=True)
        out = os.path.join(ROOT, "ab", "libkca_kernels_stamps.so")
    if ab_define:
        os.makedirs(os.path.join(ROOT, "ab"), exist_ok=True)
        out = os.path.join(ROOT, "ab", f"libkca_kernels_{ab_define.lower()}.so")
    cmd = [HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", out + ".tmp"] + objs + [
        f"-L{ROCM}/lib", "-lhipblaslt"]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"link failed: {' '.join(cmd)}\n{r.stderr}")
    os.replace(out + ".tmp", out)
    if verbose:
        print(f"built {out} from {len(srcs)} sources")
    return out


def build_host(jobs: int = 8, verbose: bool = False) -> str | None:
    srcs = []
    for sub in ("cpu", "io", "tokenize", "runtime"):
        srcs += _sources(sub, (".cpp",))
    if not srcs:
        return None
    hdrs = []
    for sub in ("cpu", "io", "tokenize", "runtime"):
        hdrs += _sources(sub, (".h",))
    obj_dir = os.path.join(BUILD, "host")
    os.makedirs(obj_dir, exist_ok=True)
    os.makedirs(OUT_DIR, exist_ok=True)
    cxx = shutil.which("g++") or "g++"
    flags = HOST_FLAGS + [f"-I{ROCM}/include", "-D__HIP_PLATFORM_AMD__"]
    with cf.ThreadPoolExecutor(max_workers=jobs) as ex:
        objs = list(ex.map(lambda s: _compile([cxx], s, hdrs, obj_dir, flags), srcs))
    out = os.path.join(OUT_DIR, "libkca_host.so")
    cmd = [cxx, "-shared", "-fPIC", "-fopenmp", "-o", out + ".tmp"] + objs + [
        f"-L{ROCM}/lib", "-lamdhip64", "-lssl", "-lcrypto", "-lpthread"]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"link failed: {' '.join(cmd)}\n{r.stderr}")
    os.replace(out + ".tmp", out)
    if verbose:
        print(f"built {out} from {len(srcs)} sources")
    return out


SANITIZE_FLAGS = ["-fsanitize=address,undefined", "-fno-sanitize-recover=all", "-fno-omit-frame-pointer", "-g", "-O1",
                  "-std=c++17", "-fopenmp", "-Wall", "-Wno-unused-function"]


def build_sanitize(verbose: bool = False) -> str:
    """ASan + UBSan executable of the host runtime (csrc/{cpu,io,tokenize}) and
    its harness csrc/tests/host_sanitize_main.cpp: the code that
    parses untrusted files / network bytes, instrumented as a standalone binary
    so no sanitizer runtime has to be preloaded into Python."""
    srcs = []
    for sub in ("cpu", "io", "tokenize", "runtime", "tests"):
        srcs += _sources(sub, (".cpp",))
    out_dir = os.path.join(BUILD, "sanitize")
    os.makedirs(out_dir, exist_ok=True)
    out = os.path.join(out_dir, "kca_host_sanitize")
    cxx = shutil.which("g++") or "g++"
    cmd = [cxx] + SANITIZE_FLAGS + [f"-I{ROCM}/include", "-D__HIP_PLATFORM_AMD__", "-o", out] + srcs + [
        f"-L{ROCM}/lib", f"-Wl,-rpath,{ROCM}/lib", "-lamdhip64", "-lssl", "-lcrypto", "-lpthread"]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"sanitize build failed: {' '.join(cmd)}\n{r.stderr}")
    if verbose:
        print(f"built {out}")
    return out


def build_all(jobs: int = 8, verbose: bool = False):
    return build_kernels(jobs, verbose), build_host(jobs, verbose), build_kernels(jobs, verbose, debug=True)


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("-j", "--jobs", type=int, default=min(8, os.cpu_count() or 1))
    ap.add_argument("--kernels-only", action="store_true")
    ap.add_argument("--debug", action="store_true", help="only the KCA_DASSERT debug kernel library")
    ap.add_argument("--sanitize", action="store_true", help="build + run the ASan/UBSan host harness")
    ap.add_argument("--stamps", action="store_true", help="only the attention stamp diagnostic library (ab/)")
    ap.add_argument("--ab-define", help="only an A/B kernel library built with -D<this> (ab/)")
    a = ap.parse_args()
    if a.ab_define:
        build_kernels(a.jobs, True, ab_define=a.ab_define)
        sys.exit(0)
    if a.stamps:
        build_kernels(a.jobs, True, stamps=True)
        sys.exit(0)
    if a.sanitize:
        exe = build_sanitize(True)
        sys.exit(subprocess.run([exe], env=dict(os.environ, ASAN_OPTIONS="detect_leaks=0:abort_on_error=1",
                                                UBSAN_OPTIONS="print_stacktrace=1")).returncode)
    if a.debug:
        build_kernels(a.jobs, True, debug=True)
        sys.exit(0)
    if a.kernels_only:
        build_kernels(a.jobs, True)
    else:
        build_all(a.jobs, True)
    sys.exit(0)
