#!/usr/bin/env python3
"""All-reduce latency sweep: the custom xGMI one-shot / two-shot kernels
(csrc/comm/xgmi_allreduce.hip) against RCCL, by message size (SURVEY §5.8,
BLOOM TP=8 decode all-reduces are B x 14336 bf16).

    torchrun --nproc-per-node 8 --master-addr 127.0.0.1 bench/allreduce_bench.py

``bench.py`` calls ``run_sweep`` on its ranks after the BLOOM TP phase when
N > 1, so the driver's scaling run records the crossover points the custom
all-reduce's switch (``parallel/custom_ar.py``: one-shot <= 256 KB, two-shot
<= 64 MB, RCCL above) should sit at. Rank 0 returns one record per size
(microseconds per call, median of timed repeats, every rank in lock step).
"""
from __future__ import annotations

import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch
import torch.distributed as dist

SIZES = (16 << 10, 64 << 10, 256 << 10, 1 << 20, 4 << 20, 16 << 20, 64 << 20)


def _time(fn, iters=20, warmup=3):
    for _ in range(warmup):
        fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(iters):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        fn()
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1) * 1e3)
    ts.sort()
    return ts[len(ts) // 2]


def run_sweep(sizes=SIZES, rccl: bool | None = None):
    """All ranks call this inside an initialised group (world > 1). Returns the
    records on rank 0 (None elsewhere)."""
    from kubernetes_cloud_amd.parallel.custom_ar import ONE_SHOT, TWO_SHOT, XGMIAllReduce
    world, rank = dist.get_world_size(), dist.get_rank()
    dev = torch.device("cuda", torch.cuda.current_device())
    if rccl is None:
        rccl = dist.get_backend() == "nccl"
    ar = XGMIAllReduce(None, max_bytes=max(sizes))
    out = []
    try:
        for nbytes in sizes:
            x = torch.ones(nbytes // 2, device=dev, dtype=torch.bfloat16)
            rec = {"bytes": nbytes, "world": world}
            for name, algo in (("one_shot_us", ONE_SHOT), ("two_shot_us", TWO_SHOT)):
                dist.barrier()
                rec[name] = round(_time(lambda: ar.all_reduce_(x, algo=algo)), 1)
            if rccl:
                dist.barrier()
                rec["rccl_us"] = round(_time(lambda: dist.all_reduce(x)), 1)
            ar.check()
            best = min((v, k) for k, v in rec.items() if k.endswith("_us"))[1]
            rec["best"] = best[:-3]
            rec["busbw_gbps_best"] = round(2 * (world - 1) / world * nbytes / rec[best] / 1e3, 1)
            out.append(rec)
    finally:
        dist.barrier()
        ar.close()
    return out if rank == 0 else None


def main():
    from kubernetes_cloud_amd.parallel.dist import init_distributed
    init_distributed()
    recs = run_sweep()
    for r in recs or ():
        print(json.dumps(r), flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
