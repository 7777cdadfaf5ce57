"""Localise errors of the tiled attention fast path vs the fp32 reference."""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch
from kubernetes_cloud_amd import ops

torch.manual_seed(0)
for D in (256,):
    for causal in (False, True):
        for Sk in (32, 64, 128):
            B, Sq, H = 1, 128, 1
            if causal and Sk < Sq:
                continue
            q = torch.randn(B, Sq, H, D, device="cuda", dtype=torch.bfloat16)
            k = torch.randn(B, Sk, H, D, device="cuda", dtype=torch.bfloat16)
            v = torch.randn(B, Sk, H, D, device="cuda", dtype=torch.bfloat16)
            o = ops.flash_attention(q, k, v, causal=causal).float()
            r, _ = ops.attention_reference(q.float(), k.float(), v.float(), causal)
            err = (o - r).abs()[0, :, 0]  # [Sq, D]
            print(f"D{D} causal={causal} Sk={Sk} max={err.max():.3f}")
            rows = err.max(1).values
            bad_rows = (rows > 0.05).nonzero().flatten().tolist()
            print("  bad rows:", bad_rows[:40], len(bad_rows))
            cols = err.max(0).values
            bad_cols = (cols > 0.05).nonzero().flatten().tolist()
            print("  bad cols:", bad_cols[:64], len(bad_cols))
            # try V = identity-ish to find which key index maps
