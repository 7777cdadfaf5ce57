#!/usr/bin/env python3
"""Build the native libraries of kubernetes_cloud_amd in-tree.

* ``libkca_kernels.so`` -- every ``csrc/kernels/*.hip`` compiled by ``hipcc
  --offload-arch=gfx950`` (CDNA4 only; no other targets, no hipify step).
* ``libkca_host.so``    -- host-side C++ runtime pieces (``csrc/cpu``,
  ``csrc/io``, ``csrc/tokenize``): AVX-512/AVX2 AdamW for offload, the
  ``.tensors`` weight streamer and the BPE tokenizer / context packer.

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


def build_kernels(jobs: int = 8, verbose: bool = False) -> str:
    srcs = _sources("kernels", (".hip",)) + _sources("comm", (".hip",))
    hdrs = _sources("kernels", (".h",)) + _sources("comm", (".h",))
    obj_dir = os.path.join(BUILD, "kernels")
    os.makedirs(obj_dir, exist_ok=True)
    os.makedirs(OUT_DIR, exist_ok=True)
    with cf.ThreadPoolExecutor(max_workers=jobs) as ex:
        objs = list(ex.map(lambda s: _compile([HIPCC], s, hdrs, obj_dir, HIP_FLAGS), srcs))
    out = os.path.join(OUT_DIR, "libkca_kernels.so")
    cmd = [HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", out + ".tmp"] + objs
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"link failed: {' '.join(cmd)}\n{r.stderr}")
    os.replace(out + ".tmp", out)
    if verbose:
        print(f"built {out} from {len(srcs)} sources")
    return out


def build_host(jobs: int = 8, verbose: bool = False) -> str | None:
    srcs = []
    for sub in ("cpu", "io", "tokenize"):
        srcs += _sources(sub, (".cpp",))
    if not srcs:
        return None
    hdrs = []
    for sub in ("cpu", "io", "tokenize"):
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


def build_all(jobs: int = 8, verbose: bool = False):
    return build_kernels(jobs, verbose), build_host(jobs, verbose)


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("-j", "--jobs", type=int, default=min(8, os.cpu_count() or 1))
    ap.add_argument("--kernels-only", action="store_true")
    a = ap.parse_args()
    if a.kernels_only:
        build_kernels(a.jobs, True)
    else:
        build_all(a.jobs, True)
    sys.exit(0)
