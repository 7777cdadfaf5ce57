#!/usr/bin/env python3
"""Decode-engine benchmark (FasterTransformer-equivalent path).

GPT-J-6B (random init, bf16) through ``LLMEngine`` with HIP-graph decode:
prefill ms, decode ms/step and generated tokens/s at several batch sizes
(FT config: request_output_len 64; download-weights-job-gptj.yml). One JSON
line per batch size.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch


SAMPLING = {
    "greedy": dict(do_sample=False),
    # the FasterTransformer GPT-J request (online-inference/fastertransformer: runtime_top_k 10,
    # temperature 1.0): sampled on the device inside the decode graph
    "ft_topk10": dict(do_sample=True, temperature=1.0, top_k=10, top_p=1.0, seed=1),
}


def run_decode(model="gpt-j-6b", batches=(1, 32), prompt_len=512, new_tokens=64, sampling=("greedy",),
               dtype="bf16"):
    """bench.py's ``secondary_decode``: per batch size and sampling mode, prefill ms and pure
    decode ms/token (HIP graphs, all requests running) -- the FT GPT-J
    serving row (request_output_len 64). ``dtype`` "fp16": FT's ``data_type: fp16`` (the native
    fp16 decode step: matrix-core layer at every batch)."""
    from kubernetes_cloud_amd.engine.llm_engine import LLMEngine, SamplingParams
    from kubernetes_cloud_amd.models.causal_lm import build_model
    from kubernetes_cloud_amd.models.config import preset
    dev = torch.device("cuda", torch.cuda.current_device())
    cfg = preset(model)
    m = build_model(cfg, device=dev, dtype={"bf16": torch.bfloat16, "fp16": torch.float16}[dtype], seed=0)
    m.eval()
    eng = LLMEngine(m, max_slots=max(batches), max_len=prompt_len + new_tokens + 16)
    g = torch.Generator().manual_seed(0)
    out = []
    for B, mode in ((b, s) for b in batches for s in sampling):
        prompts = [torch.randint(0, cfg.vocab_size, (prompt_len,), generator=g).tolist() for _ in range(B)]
        sp = SamplingParams(max_new_tokens=new_tokens, **SAMPLING[mode])
        eng.generate(prompts, sp)  # warm-up + graph capture for this bucket
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        eng.runner.prefill(torch.tensor(prompts[:1]), [0])
        torch.cuda.synchronize()
        prefill_ms = (time.perf_counter() - t0) * 1e3
        eng.runner.release(0)
        reqs = [eng.add_request(p, sp) for p in prompts]
        eng.step()  # admit (prefill + first token) + first decode
        torch.cuda.synchronize()
        s0, t0 = eng.stats["decode_steps"], time.perf_counter()
        eng.run_until_done(reqs)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        n = eng.stats["decode_steps"] - s0
        out.append({"metric": f"{model} decode", "batch": B, "sampling": mode, "prompt_len": prompt_len,
                    "new_tokens": new_tokens,
                    "prefill_ms_one_seq": round(prefill_ms, 2), "decode_ms_per_token": round(dt / max(n, 1) * 1e3, 3),
                    "decode_tokens_per_s": round(B * n / dt, 1), "dtype": dtype, "graphs": eng.runner.use_graphs,
                    "data": "random-init weights, random prompts"})
    del eng, m
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="gpt-j-6b")
    ap.add_argument("--batches", default="1,8,32,64")
    ap.add_argument("--prompt-len", type=int, default=512)
    ap.add_argument("--new-tokens", type=int, default=64)
    ap.add_argument("--layers", type=int, default=0, help="override layer count (smoke runs only)")
    ap.add_argument("--no-graphs", action="store_true")
    ap.add_argument("--page-size", type=int, default=None, help="KV page size (0 = contiguous slots)")
    ap.add_argument("--decode-only", type=int, default=0,
                    help="profile mode: prefill B prompts once, then time N pure decode steps")
    ap.add_argument("--tune", default=None,
                    help="TunableOp: search the GEMM solutions of this run and write them to this file "
                         "(run with --no-graphs; graphs cannot capture the search)")
    args = ap.parse_args()
    if args.tune:
        os.environ["KCA_TUNABLEOP"] = "off"  # no preloaded table: search everything this run touches
        from kubernetes_cloud_amd.utils import tunable
        tunable.configure(args.tune, "tune", max_tuning_ms=30)
    from kubernetes_cloud_amd.engine.llm_engine import LLMEngine, SamplingParams
    from kubernetes_cloud_amd.models.causal_lm import build_model
    from kubernetes_cloud_amd.models.config import preset
    from kubernetes_cloud_amd.ops import _lib
    _lib.require()
    dev = torch.device("cuda", 0)
    cfg = preset(args.model)
    if args.layers:
        cfg.n_layers = args.layers
    m = build_model(cfg, device=dev, dtype=torch.bfloat16, seed=0)
    batches = [int(b) for b in args.batches.split(",")]
    # (decode-only: room for every timed step -- a request that hit max_len would leave the
    # remaining steps empty and the average meaningless)
    eng = LLMEngine(m, max_slots=max(batches), max_len=args.prompt_len + max(args.new_tokens, args.decode_only) + 16,
                    use_graphs=not args.no_graphs, page_size=args.page_size)
    g = torch.Generator().manual_seed(0)
    if args.decode_only:
        B = batches[0]
        prompts = [torch.randint(0, cfg.vocab_size, (args.prompt_len,), generator=g).tolist() for _ in range(B)]
        sp = SamplingParams(max_new_tokens=args.decode_only + 8, do_sample=False)
        reqs = [eng.add_request(p, sp) for p in prompts]
        for _ in range(4):
            eng.step()  # admit + warm the graph bucket
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(args.decode_only):
            eng.step()
        torch.cuda.synchronize()
        assert all(not r.done for r in reqs), "a request finished inside the timed decode-only steps"
        dt = (time.perf_counter() - t0) / args.decode_only
        print(json.dumps({"metric": f"{args.model} decode-only", "batch": B, "decode_ms_per_step": round(dt * 1e3, 3),
                          "decode_tokens_per_s": round(B / dt, 1), "page_size": eng.runner.cache.page_size}),
              flush=True)
        return
    for B in batches:
        prompts = [torch.randint(0, cfg.vocab_size, (args.prompt_len,), generator=g).tolist() for _ in range(B)]
        sp = SamplingParams(max_new_tokens=args.new_tokens, temperature=1.0, top_k=50, top_p=0.95, seed=1)
        eng.generate(prompts, SamplingParams(max_new_tokens=args.new_tokens, do_sample=False))  # warm/capture
        torch.cuda.synchronize()
        # prefill alone
        t0 = time.perf_counter()
        for p in prompts:
            eng.runner.prefill(torch.tensor([p]), [0])
        torch.cuda.synchronize()
        eng.runner.release(0)
        prefill_ms = (time.perf_counter() - t0) / B * 1e3
        reqs = [eng.add_request(p, sp) for p in prompts]
        eng.step()  # admit + first decode
        torch.cuda.synchronize()
        steps0, t0 = eng.stats["decode_steps"], time.perf_counter()
        eng.run_until_done(reqs)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        nsteps = eng.stats["decode_steps"] - steps0
        gen = sum(len(r.output) for r in reqs) - 2 * B
        print(json.dumps({"metric": f"{args.model} decode", "batch": B, "prompt_len": args.prompt_len,
                          "new_tokens": args.new_tokens, "prefill_ms_per_seq": round(prefill_ms, 2),
                          "decode_ms_per_step": round(dt / max(nsteps, 1) * 1e3, 3),
                          "decode_tokens_per_s": round(gen / dt, 1), "graphs": not args.no_graphs,
                          "kv_cache_gib": round(eng.runner.cache.nbytes() / 2**30, 2),
                          "page_size": eng.runner.cache.page_size,
                          "layers": cfg.n_layers}), flush=True)


if __name__ == "__main__":
    main()
