#!/usr/bin/env python3
"""Time the SD-1.5 txt2img pieces separately on the GPU (text encoder, one
CFG UNet step through the HIP-graph runner, VAE decode of the batch) so the
images/s number in bench.py can be attributed.  ``--only vae`` runs just the
decode (for a kernel trace of the VAE)."""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "bench"))

import torch  # noqa: E402


def timed(fn, iters):
    fn()
    torch.cuda.synchronize()
    time.sleep(1.0)  # idle gap: marks the start of the steady-state dispatches in a kernel trace
    t = time.perf_counter()
    for _ in range(iters):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / iters * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=8)
    ap.add_argument("--only", default="")
    ap.add_argument("--iters", type=int, default=3)
    args = ap.parse_args()
    from sd_bench import build
    from kubernetes_cloud_amd.models.sd_pipeline import unet_runner

    dev = torch.device("cuda", 0)
    unet, vae, te = build(dev, torch.bfloat16)
    for m in (unet, vae, te):
        m.eval()
    B = args.batch
    z = torch.randn(B, 4, 64, 64, device=dev, dtype=torch.bfloat16)
    out = {}
    with torch.no_grad():
        if args.only in ("", "vae"):
            out["vae_decode_ms"] = timed(lambda: vae.decode(z), args.iters)
        if args.only in ("", "unet"):
            ids = torch.randint(0, 49408, (2 * B, 77), device=dev)
            out["text_encoder_ms"] = timed(lambda: te(ids), args.iters)
            ctx = te(ids)
            run_unet = unet_runner(unet)
            xin = torch.randn(2 * B, 4, 64, 64, device=dev, dtype=torch.bfloat16)
            tt = torch.full((2 * B,), 500.0, device=dev)
            out["unet_step_ms"] = timed(lambda: run_unet(xin, tt, ctx), 10)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
