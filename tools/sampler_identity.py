#!/usr/bin/env python3
"""Sampler A/B identity: the same logits, seeds and settings through the library this process loaded
(KCA_KERNEL_LIB selects it), written to ``--out``; ``--compare A B`` then checks that two runs drew
the same ids and kept-set sizes. Used when a sampler change must not change a single draw.

    KCA_KERNEL_LIB=$PWD/ab/libkca_kernels_old.so python tools/sampler_identity.py --out gpurun_out/old.pt
    python tools/sampler_identity.py --out gpurun_out/new.pt
    python tools/sampler_identity.py --compare gpurun_out/old.pt gpurun_out/new.pt
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

MODES = {"greedy": (0.0, 0, 1.0), "topk10": (1.0, 10, 1.0), "topk50": (1.0, 50, 1.0),
         "topk50_topp0.95": (1.0, 50, 0.95), "topp0.95": (1.0, 0, 0.95), "topk64_t0.7_topp0.8": (0.7, 64, 0.8),
         "topk1": (1.0, 1, 1.0), "topk20_topp0.5": (1.3, 20, 0.5)}


def run(out):
    from kubernetes_cloud_amd.ops import decode as dops
    dev = torch.device("cuda", 0)
    res = {}
    for V in (50400, 250880):
        g = torch.Generator(device=dev).manual_seed(V)
        B = 64
        dists = {
            "randn4": torch.randn(B, V, device=dev, generator=g) * 4,
            "randn05": torch.randn(B, V, device=dev, generator=g) * 0.5,
            "ties": torch.randint(0, 12, (B, V), device=dev, generator=g).float(),
        }
        for dn, lg in dists.items():
            lg = lg.to(torch.bfloat16)
            for mn, (t, k, p) in MODES.items():
                f = lambda v, dt: torch.full((B,), v, dtype=dt, device=dev)  # noqa: E731
                kept = torch.empty(B, dtype=torch.int32, device=dev)
                ids, lp = dops.sample_logits(lg, temperature=f(t, torch.float32), top_k=f(k, torch.int32),
                                             top_p=f(p, torch.float32), rep_penalty=f(1.0, torch.float32),
                                             seeds=torch.arange(B, device=dev) * 7919 + 1, out_kept=kept)
                res[f"{V}/{dn}/{mn}"] = (ids.cpu(), kept.cpu(), lp.cpu())
    torch.save(res, out)
    print(f"wrote {len(res)} cases to {out}")


def compare(a, b):
    ra, rb = torch.load(a, weights_only=True), torch.load(b, weights_only=True)
    bad = 0
    for key in ra:
        ia, ka, la = ra[key]
        ib, kb, lb = rb[key]
        same = torch.equal(ia, ib) and torch.equal(ka, kb) and torch.equal(la, lb)
        if not same:
            bad += 1
            print(f"DIFF {key}: ids {int((ia != ib).sum())} kept {int((ka != kb).sum())}")
    print(f"{len(ra) - bad}/{len(ra)} cases identical")
    return bad == 0


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--out")
    ap.add_argument("--compare", nargs=2)
    a = ap.parse_args()
    if a.compare:
        sys.exit(0 if compare(*a.compare) else 1)
    run(a.out)
