"""GPU check: SD BasicTransformerBlock with the residual adds fused into the
following LayerNorm, forward+backward twice (anomaly mode names a failing node)."""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch
from kubernetes_cloud_amd.models.unet import BasicTransformerBlock
torch.autograd.set_detect_anomaly(True)
dev = "cuda"
blk = BasicTransformerBlock(320, 8, 40, 64).to(dev, torch.bfloat16)
x = torch.randn(2, 256, 320, device=dev, dtype=torch.bfloat16, requires_grad=True)
ctx = torch.randn(2, 7, 64, device=dev, dtype=torch.bfloat16)
for i in range(2):
    y = blk(x, ctx)
    y.float().square().mean().backward()
    print("iter", i, "ok", flush=True)
