#!/usr/bin/env python3
"""TunableOp search for the BLOOM-176B tensor-parallel serving GEMMs on one MI355X.

The per-rank shard GEMMs of BLOOM-176B at TP = 2 / 4 / 8 (the ranks of the driver's multi-GPU
bench and the bloom-176b-deepspeed service) at decode batch buckets that reach hipBLASLt
(M = 4 ... 64; M = 1 and 2 stream through the GEMV kernels) and prefill row counts, called
through F.linear exactly as engine/runner.py does (column-parallel with bias, row-parallel
without: the bias follows the all-reduce). Results merge into a copy of
tuning/tunableop_decode.csv written under --out; copy it back to tuning/ afterwards.

    python tools/tune_bloom_tp_gemms.py --out gpurun_out/tunableop_decode.csv
"""
from __future__ import annotations

import argparse
import os
import shutil
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", required=True)
    ap.add_argument("--tps", default="2,4,8")
    ap.add_argument("--ms", default="4,8,16,32,64,128,1024,4096")
    ap.add_argument("--max-ms", type=int, default=30)
    a = ap.parse_args()
    from kubernetes_cloud_amd.utils import tunable as kt
    os.makedirs(os.path.dirname(os.path.abspath(a.out)), exist_ok=True)
    if os.path.exists(kt.DECODE_FILE) and not os.path.exists(a.out):
        shutil.copy(kt.DECODE_FILE, a.out)
    import torch
    import torch.nn.functional as F
    kt.configure(a.out, "tune", max_tuning_ms=a.max_ms)
    dev = torch.device("cuda", 0)
    d, ffn, vocab = 14336, 4 * 14336, 250880
    t0 = time.time()
    n = 0
    for tp in (int(x) for x in a.tps.split(",")):
        shapes = [(3 * d // tp, d, True), (d, d // tp, False), (ffn // tp, d, True), (d, ffn // tp, False),
                  (vocab // tp, d, False)]
        for (N, K, bias) in shapes:
            w = torch.randn(N, K, device=dev, dtype=torch.bfloat16) * 0.01
            b = torch.randn(N, device=dev, dtype=torch.bfloat16) if bias else None
            for M in (int(x) for x in a.ms.split(",")):
                if N == vocab // tp and M > 64:
                    continue  # the LM head only sees the last position of each sequence
                x = torch.randn(M, K, device=dev, dtype=torch.bfloat16)
                F.linear(x, w, b)
                torch.cuda.synchronize()
                n += 1
            print(f"[tune] tp={tp} N={N} K={K} bias={bias} done ({n} shapes, {time.time() - t0:.0f}s)",
                  flush=True)
            del w, b
    print(f"[tune] {n} shapes; TunableOp writes {a.out} at exit", flush=True)


if __name__ == "__main__":
    main()
