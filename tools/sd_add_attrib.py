#!/usr/bin/env python3
"""Attribute the SD UNet's elementwise add kernels to their call sites: one eager UNet forward
(txt2img shape: batch 16, 64x64 latent) under torch.profiler with shapes, aten::add / add_ /
convolution entries grouped by input shapes."""
import collections
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import importlib.util

import torch

spec = importlib.util.spec_from_file_location("sdb", os.path.join(os.path.dirname(os.path.dirname(
    os.path.abspath(__file__))), "bench", "sd_bench.py"))
sdb = importlib.util.module_from_spec(spec)
spec.loader.exec_module(sdb)
from kubernetes_cloud_amd.utils import miopen  # noqa: E402

miopen.configure()
dev = torch.device("cuda", 0)
unet, vae, te = sdb.build(dev, torch.bfloat16)
unet.eval()
x = torch.randn(16, 4, 64, 64, device=dev, dtype=torch.bfloat16).to(memory_format=torch.channels_last)
ctx = torch.randn(16, 77, 768, device=dev, dtype=torch.bfloat16)
t = torch.full((16,), 500.0, device=dev)
with torch.no_grad():
    for _ in range(2):
        unet(x, t, ctx)
    torch.cuda.synchronize()
    from torch.profiler import ProfilerActivity, profile
    with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], record_shapes=True) as prof:
        unet(x, t, ctx)
        torch.cuda.synchronize()
agg = collections.Counter()
for ev in prof.events():
    if ev.name in ("aten::add", "aten::add_", "aten::convolution", "aten::addmm", "aten::mul"):
        agg[(ev.name, str(ev.input_shapes)[:140])] += 1
for (n, sh), c in sorted(agg.items(), key=lambda kv: -kv[1])[:40]:
    print(c, n, sh)
print(prof.key_averages().table(sort_by="cuda_time_total", row_limit=25))
