#!/usr/bin/env python3
"""A/B of bf16 transpose kernel variants (csrc/ab/transpose_ab.hip) and the
shipping GELU-transpose tile kernels at the GPT-J training shapes: achieved
GB/s of compulsory HBM bytes, with a rotation of 4 buffer sets (> the 256 MB
MALL) so every call streams from HBM."""
import ctypes
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
lib = ctypes.CDLL(os.path.join(ROOT, "ab", "libkca_transpose_ab.so"))
lib.ab_transpose.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_longlong, ctypes.c_void_p, ctypes.c_longlong,
                             ctypes.c_int, ctypes.c_int, ctypes.c_void_p]


def timeit(fn, sets, n=12):
    for i in range(4):
        fn(sets[i % len(sets)])
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for i in range(n):
        fn(sets[i % len(sets)])
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / n


def main():
    from kubernetes_cloud_amd.ops import _lib
    kl = _lib.require()
    st = lambda: torch.cuda.current_stream().cuda_stream  # noqa: E731
    shapes = [(16384, 4096), (16384, 16384), (32768, 4096)]
    variants = [int(a) for a in (sys.argv[1].split(",") if len(sys.argv) > 1 else "9,0,1,2,3,5,6".split(","))]
    for R, C in shapes:
        nset = 4
        sets = [(torch.randn(R, C, device="cuda").to(torch.bfloat16), torch.empty(C, R, device="cuda", dtype=torch.bfloat16),
                 torch.empty(R, C, device="cuda", dtype=torch.bfloat16),
                 torch.randn(R, C, device="cuda").to(torch.bfloat16)) for _ in range(nset)]
        x, y = sets[0][0], sets[0][1]
        ref = x.t().contiguous()
        for v in variants:
            def f(s, v=v):
                assert lib.ab_transpose(v, s[0].data_ptr(), C, s[1].data_ptr(), R, R, C, st()) == 0
            if v != 9:
                y.zero_()
                f(sets[0])
                torch.cuda.synchronize()
                assert torch.equal(y, ref), (v, R, C)
            ms = timeit(f, sets)
            print(json.dumps({"R": R, "C": C, "kernel": f"transpose_v{v}" if v != 9 else "copy", "ms": round(ms, 4),
                              "gbps": round(2 * R * C * 2 / ms / 1e6, 1), "sets": nset}), flush=True)
        # shipping fused kernels: gelu fwd (read h, write g + g^T), gelu bwd (read dg + h, write dh + dh^T)
        def gf(s):
            assert kl.kca_gelu_fwd_t(ctypes.c_void_p(s[0].data_ptr()), ctypes.c_longlong(C),
                                     ctypes.c_void_p(s[2].data_ptr()), ctypes.c_longlong(C),
                                     ctypes.c_void_p(s[1].data_ptr()), ctypes.c_longlong(R), R, C, 1,
                                     ctypes.c_void_p(st())) == 0
        ms = timeit(gf, sets)
        print(json.dumps({"R": R, "C": C, "kernel": "gelu_fwd_t", "ms": round(ms, 4),
                          "gbps": round(3 * R * C * 2 / ms / 1e6, 1)}), flush=True)

        def gb(s):
            assert kl.kca_gelu_bwd_t(ctypes.c_void_p(s[0].data_ptr()), ctypes.c_longlong(C),
                                     ctypes.c_void_p(s[3].data_ptr()), ctypes.c_longlong(C),
                                     ctypes.c_void_p(s[2].data_ptr()), ctypes.c_longlong(C),
                                     ctypes.c_void_p(s[1].data_ptr()), ctypes.c_longlong(R), None, R, C, 1,
                                     ctypes.c_void_p(st())) == 0
        ms = timeit(gb, sets)
        print(json.dumps({"R": R, "C": C, "kernel": "gelu_bwd_t", "ms": round(ms, 4),
                          "gbps": round(4 * R * C * 2 / ms / 1e6, 1)}), flush=True)
        del sets
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
