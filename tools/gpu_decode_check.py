#!/usr/bin/env python3
"""Decode numbers of bench.py's extra records, alone: GPT-J-6B and GPT-NeoX-20B (B = 1 / 32, greedy and
top-k 10) and BLOOM-176B TP=8 rank-0 emulation (B = 1 / 8 / 32). One JSON line per record group."""
import importlib.util
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402


def _load(name):
    spec = importlib.util.spec_from_file_location(f"kca_{name}", os.path.join(ROOT, "bench", f"{name}.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def main():
    which = sys.argv[1:] or ["gptj", "neox", "bloom"]
    db = _load("decode_bench")
    if "gptj" in which:
        print(json.dumps({"gptj": db.run_decode("gpt-j-6b", batches=(1, 32), prompt_len=512, new_tokens=64,
                                                sampling=("greedy", "ft_topk10"))}), flush=True)
        torch.cuda.empty_cache()
    if "neox" in which:
        print(json.dumps({"neox": db.run_decode("gpt-neox-20b", batches=(1, 32), prompt_len=512, new_tokens=64,
                                                sampling=("greedy", "ft_topk10"))}), flush=True)
        torch.cuda.empty_cache()
    if "bloom" in which:
        recs = _load("bloom_tp_bench").run_tp_decode("bloom-176b", layers=0, batches=(1, 8, 32), prompt_len=128,
                                                     new_tokens=32, emulate_tp=8)
        print(json.dumps({"bloom_tp8_rank": recs}), flush=True)


if __name__ == "__main__":
    main()
