#!/usr/bin/env python3
"""DALL·E mini / mega text-to-image latency on one MI355X (S12): random-init
weights of the published architectures (no network for checkpoints), 256 image
tokens with super conditioning (batch 2 internally), VQGAN f16 decode to
256x256, PNG encode excluded."""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", choices=["mini", "mega"], default="mini")
    ap.add_argument("--images", type=int, default=2)
    args = ap.parse_args()
    from kubernetes_cloud_amd.models.dalle_mini import DalleBartConfig
    from kubernetes_cloud_amd.ops import _lib
    from kubernetes_cloud_amd.serving.dalle_service import DalleMiniPredictor, options
    _lib.require()
    cfg = DalleBartConfig.mega() if args.model == "mega" else DalleBartConfig()
    p = DalleMiniPredictor(f"dalle-{args.model}", None, options({}), device=torch.device("cuda", 0), config=cfg)
    p.load()
    prm = p.configure_request({"parameters": {}})
    p.generate_images(["warmup"], prm, seed=0)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(args.images):
        img = p.generate_images(["an armchair in the shape of an avocado"], prm, seed=i)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / args.images
    n = sum(x.numel() for x in p.model.parameters())
    print(json.dumps({"metric": f"dalle-{args.model} text-to-image", "s_per_image": round(dt, 3),
                      "images_per_s": round(1 / dt, 3), "params": n, "image_tokens": cfg.image_length,
                      "condition_scale": prm["CONDITION_SCALE"], "out_shape": list(img.shape), "dtype": "bf16"}),
          flush=True)


if __name__ == "__main__":
    main()
