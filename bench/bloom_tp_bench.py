#!/usr/bin/env python3
"""BLOOM-176B TP inference benchmark (BASELINE config 4).

    torchrun --nproc-per-node 8 --master-addr 127.0.0.1 bench/bloom_tp_bench.py
    python bench/bloom_tp_bench.py --layers 8          # 1-GPU smoke (TP=1, 8 of 70 layers)

Random-init BLOOM weights (no checkpoint offline), bf16, sharded over the
launch's ranks with ``parallel.tensor_parallel`` (2 RCCL all-reduces per layer
over xGMI). Reports prefill ms (prompt 128), decode ms/token and generated
tokens/s at batch 1/8/32 through the same lock-stepped engine the TP server
uses. Rank 0 prints one JSON line per batch size.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch
import torch.distributed as dist


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="bloom-176b")
    ap.add_argument("--layers", type=int, default=0)
    ap.add_argument("--batches", default="1,8,32")
    ap.add_argument("--prompt-len", type=int, default=128)
    ap.add_argument("--new-tokens", type=int, default=64)
    args = ap.parse_args()
    from kubernetes_cloud_amd.engine.llm_engine import LLMEngine, SamplingParams
    from kubernetes_cloud_amd.engine.runner import ModelRunner
    from kubernetes_cloud_amd.engine.tp_driver import CollectiveRunner, follower_loop
    from kubernetes_cloud_amd.models.config import preset
    from kubernetes_cloud_amd.ops import _lib
    from kubernetes_cloud_amd.parallel.dist import init_distributed
    from kubernetes_cloud_amd.parallel.tensor_parallel import load_tp_model
    _lib.require()
    info = init_distributed()
    rank, world = info.rank, info.world_size
    ctrl = dist.new_group(backend="gloo") if world > 1 else None
    cfg = preset(args.model)
    if args.layers:
        cfg.n_layers = args.layers
    dev = torch.device("cuda", torch.cuda.current_device())
    t0 = time.perf_counter()
    if world > 1:
        model = load_tp_model(cfg, rank, world, None, device=dev, dtype=torch.bfloat16, random_init=True)
    else:
        from kubernetes_cloud_amd.models.causal_lm import build_model
        model = build_model(cfg, device=dev, dtype=torch.bfloat16, seed=0)
    torch.cuda.synchronize()
    load_s = time.perf_counter() - t0
    batches = [int(b) for b in args.batches.split(",")]
    if world > 1:  # one-shot xGMI all-reduce for the decode-size TP reductions
        from kubernetes_cloud_amd.parallel.custom_ar import register
        register(None)
    runner = ModelRunner(model, max_slots=max(batches), max_len=args.prompt_len + args.new_tokens + 8)
    if rank != 0:
        follower_loop(runner, ctrl)
        dist.barrier()
        return
    run = CollectiveRunner(runner, ctrl) if world > 1 else runner
    eng = LLMEngine(model, runner=run)
    g = torch.Generator().manual_seed(0)
    for B in batches:
        prompts = [torch.randint(0, cfg.vocab_size, (args.prompt_len,), generator=g).tolist() for _ in range(B)]
        sp = SamplingParams(max_new_tokens=args.new_tokens, do_sample=False)
        eng.generate(prompts, sp)  # warm-up + graph capture for this bucket
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        run.prefill(torch.tensor(prompts[:1]), [0])
        torch.cuda.synchronize()
        prefill_ms = (time.perf_counter() - t0) * 1e3
        reqs = [eng.add_request(p, sp) for p in prompts]
        eng.step()
        torch.cuda.synchronize()
        s0, t0 = eng.stats["steps"], time.perf_counter()
        eng.run_until_done(reqs)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        n = eng.stats["steps"] - s0
        print(json.dumps({"metric": f"{args.model} TP={world} decode", "batch": B, "prompt_len": args.prompt_len,
                          "prefill_ms": round(prefill_ms, 2), "decode_ms_per_token": round(dt / max(n, 1) * 1e3, 3),
                          "tokens_per_s": round((sum(len(r.output) for r in reqs) - 2 * B) / dt, 1),
                          "layers": cfg.n_layers, "tp": world, "load_s": round(load_s, 1), "dtype": "bf16",
                          "data": "random-init weights"}), flush=True)
    if world > 1:
        run.shutdown()
        dist.barrier()


if __name__ == "__main__":
    main()
