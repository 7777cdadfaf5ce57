"""HostOffloadAdamW vs FlatAdamW on GPU buffers: locate the first diverging chunk."""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch
from kubernetes_cloud_amd.train.optim import FlatAdamW, HostOffloadAdamW

torch.manual_seed(0)
n = 64 * 5000
dev = "cuda"
p0 = torch.randn(n, device=dev)
mask = (torch.arange(n // 64, device=dev) % 2).to(torch.uint8)
bf = [torch.empty(n, device=dev, dtype=torch.bfloat16) for _ in range(2)]
HostOffloadAdamW.CHUNK = 64 * 700
a = FlatAdamW(p0.clone(), lr=1e-2, weight_decay=0.1, wd_mask=mask, model_bf16=bf[0])
b = HostOffloadAdamW(p0.clone(), lr=1e-2, weight_decay=0.1, wd_mask=mask, model_bf16=bf[1])
for it in range(3):
    g = torch.randn(n, device=dev)
    a.grad.copy_(g)
    b.grad.copy_(g)
    for o in (a, b):
        o.set_clip(o.local_sumsq(), 1.0)
        o.step(use_clip=True)
    torch.cuda.synchronize()
    d = (a.master.cpu() - b.master).abs()
    bad = (d > 1e-4).nonzero().flatten()
    print("iter", it, "max diff", float(d.max()), "first bad", bad[:5].tolist(), "count", bad.numel())
    db = (bf[0].float() - bf[1].float()).abs()
    print("   bf16 max diff", float(db.max()), "first bad", (db > 1e-2).nonzero().flatten()[:5].tolist())
