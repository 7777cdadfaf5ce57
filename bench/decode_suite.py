#!/usr/bin/env python3
"""The decode rows of BASELINE config 4 / the FT services in one process (same-box A/B of a decode
change): GPT-J-6B and GPT-NeoX-20B ms/token at the given batches (bench/decode_bench.py run_decode)
and rank 0 of BLOOM-176B TP=8 (bench/bloom_tp_bench.py run_tp_decode, emulated collectives).

    python bench/decode_suite.py --models gptj,neox,bloom8 --batches 1,8,32
    KCA_DECODE_FUSED_BATCHED=0 python bench/decode_suite.py ...   # the per-projection batch > 1 path
One JSON line per record.
"""
from __future__ import annotations

import argparse
import importlib.util
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def _load(name):
    spec = importlib.util.spec_from_file_location(f"kca_{name}", os.path.join(ROOT, "bench", f"{name}.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--models", default="gptj,neox,bloom8")
    ap.add_argument("--batches", default="1,8,32")
    ap.add_argument("--sampling", default="greedy")
    ap.add_argument("--new-tokens", type=int, default=64)
    ap.add_argument("--dtypes", default="bf16", help="comma list of bf16 / fp16")
    args = ap.parse_args()
    import torch
    batches = tuple(int(b) for b in args.batches.split(","))
    tag = {"batched_fused": os.environ.get("KCA_DECODE_FUSED_BATCHED", "1")}
    for name, dt in ((n, d) for n in args.models.split(",") for d in args.dtypes.split(",")):
        if name in ("gptj", "neox"):
            model = {"gptj": "gpt-j-6b", "neox": "gpt-neox-20b"}[name]
            recs = _load("decode_bench").run_decode(model, batches=batches, prompt_len=512,
                                                    new_tokens=args.new_tokens,
                                                    sampling=tuple(args.sampling.split(",")), dtype=dt)
        elif name == "bloom8":
            recs = _load("bloom_tp_bench").run_tp_decode("bloom-176b", layers=0, batches=batches, prompt_len=128,
                                                         new_tokens=32, emulate_tp=8, dtype=dt)
        else:
            raise ValueError(name)
        for r in recs:
            r.update(tag)
            print(json.dumps(r), flush=True)
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
