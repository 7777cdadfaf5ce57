#!/usr/bin/env python3
"""SD-1.5 UNet training step (DreamBooth shape: 16 x 64x64 latents) under torch.profiler: CUDA
time of every GEMM (aten::mm / addmm / bmm) grouped by input shapes -- finds the small-output,
long-K weight-gradient GEMMs."""
import collections
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import importlib.util

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
spec = importlib.util.spec_from_file_location("sdb", os.path.join(ROOT, "bench", "sd_bench.py"))
sdb = importlib.util.module_from_spec(spec)
spec.loader.exec_module(sdb)
from kubernetes_cloud_amd.utils import miopen, tunable  # noqa: E402

miopen.configure()
tunable.ensure(tunable.SD_FILE)
dev = torch.device("cuda", 0)
unet, vae, te = sdb.build(dev, torch.bfloat16)
unet.train()
x = torch.randn(16, 4, 64, 64, device=dev, dtype=torch.bfloat16).to(memory_format=torch.channels_last)
ctx = torch.randn(16, 77, 768, device=dev, dtype=torch.bfloat16)
t = torch.randint(0, 1000, (16,), device=dev)


def step():
    out = unet(x, t, ctx)
    out.float().pow(2).mean().backward()


for _ in range(2):
    step()
torch.cuda.synchronize()
from torch.profiler import ProfilerActivity, profile  # noqa: E402

with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], record_shapes=True) as prof:
    step()
    torch.cuda.synchronize()
rows = collections.defaultdict(lambda: [0, 0.0])
for e in prof.key_averages(group_by_input_shape=True):
    if e.key in ("aten::mm", "aten::addmm", "aten::bmm", "aten::matmul", "aten::convolution_backward",
                 "aten::sum", "aten::linear"):
        k = (e.key, str(e.input_shapes)[:120])
        rows[k][0] += e.count
        rows[k][1] += e.device_time_total if hasattr(e, "device_time_total") else e.cuda_time_total
tot = sum(v[1] for v in rows.values())
for (n, sh), (c, us) in sorted(rows.items(), key=lambda kv: -kv[1][1])[:35]:
    print(f"{us / 1e3:8.2f} ms {c:4d}x {n:28s} {sh}")
