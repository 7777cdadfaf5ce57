#!/usr/bin/env python3
"""BLOOM-176B TP inference benchmark (BASELINE config 4).

    torchrun --nproc-per-node 8 --master-addr 127.0.0.1 bench/bloom_tp_bench.py
    python bench/bloom_tp_bench.py --layers 8          # 1-GPU smoke (TP=1, 8 of 70 layers)

Random-init BLOOM weights (no checkpoint offline), bf16, sharded over the
launch's ranks with ``parallel.tensor_parallel`` (2 all-reduces per layer over
xGMI: the custom one-/two-shot kernel up to 64 MB, RCCL above). Reports
prefill ms (prompt 128), decode ms/token and generated tokens/s at batch
1/8/32 through the same lock-stepped engine the TP server uses. Rank 0 prints
one JSON line per batch size. ``bench.py`` calls ``run_tp_decode`` for its
secondary BLOOM measurement when it runs on more than one GPU.
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


def run_tp_decode(model_name="bloom-176b", layers=0, batches=(1, 8, 32), prompt_len=128, new_tokens=64,
                  custom_ar=True, dtype="bf16", emulate_tp=0):
    """All ranks call this inside an initialised process group (or world 1). ``dtype`` "fp16" runs
    the model in float16 as BASELINE config 4 / DS-Inference state (the native fp16 decode step: the
    same per-batch dispatch as bf16, the all-reduce tails' fp16 instantiations). ``emulate_tp`` N > 1 (one process, no process
    group): rank 0's shard of a TP=N layout with stand-in collectives (parallel/tp_emulation.py) --
    the per-rank weight stream and kernel schedule of the real run, all-reduces priced separately.
    Returns the per-batch records on rank 0, None on followers."""
    from kubernetes_cloud_amd.engine.llm_engine import LLMEngine, SamplingParams
    from kubernetes_cloud_amd.engine.runner import ModelRunner
    from kubernetes_cloud_amd.engine.tp_driver import CollectiveRunner, follower_loop
    from kubernetes_cloud_amd.models.config import preset
    from kubernetes_cloud_amd.ops import _lib
    _lib.require()
    world = dist.get_world_size() if dist.is_initialized() else 1
    rank = dist.get_rank() if dist.is_initialized() else 0
    ctrl = dist.new_group(backend="gloo") if world > 1 else None
    cfg = preset(model_name)
    if layers:
        cfg.n_layers = layers
    dev = torch.device("cuda", torch.cuda.current_device())
    tdt = {"bf16": torch.bfloat16, "fp16": torch.float16}[dtype]
    t0 = time.perf_counter()
    emu = None
    if emulate_tp > 1:
        if world > 1:
            raise ValueError("emulate_tp runs one process")
        from kubernetes_cloud_amd.parallel.tp_emulation import emulated_rank_model
        model = emulated_rank_model(cfg, emulate_tp, 0, device=dev, dtype=tdt)
        emu = model.h[0].attn.out.group
    elif dist.is_initialized():  # TP modules even at world 1: exercises the RCCL collectives in the decode graph
        from kubernetes_cloud_amd.parallel.tensor_parallel import load_tp_model
        model = load_tp_model(cfg, rank, world, None, device=dev, dtype=tdt, random_init=True)
    else:
        from kubernetes_cloud_amd.models.causal_lm import build_model
        model = build_model(cfg, device=dev, dtype=tdt, seed=0)
    torch.cuda.synchronize()
    load_s = time.perf_counter() - t0
    ar = None
    if world > 1 and custom_ar:
        from kubernetes_cloud_amd.parallel.custom_ar import register
        ar = register(None)
    elif emu is not None and custom_ar:
        # a rank-local custom all-reduce for the emulated group: the emulated rank closes each row-parallel
        # projection with the same fused all-reduce tail kernels a TP=8 rank runs (kca_ar_res_ln at batch 1,
        # kca_ar_res_stats at batch > 1), itself the only peer -- the measured step has the deployment's
        # launch structure, minus the xGMI transfers
        from kubernetes_cloud_amd.parallel.custom_ar import register
        ar = register(emu)
    runner = ModelRunner(model, max_slots=max(batches), max_len=prompt_len + new_tokens + 8)
    chan = None
    if world > 1:
        from kubernetes_cloud_amd.engine.ctrl_channel import open_channel
        chan = open_channel(ctrl)
    out = None
    if rank != 0:
        follower_loop(runner, chan)
    else:
        run = CollectiveRunner(runner, chan) if world > 1 else runner
        eng = LLMEngine(model, runner=run)
        g = torch.Generator().manual_seed(0)
        out = []
        for B in batches:
            prompts = [torch.randint(0, cfg.vocab_size, (prompt_len,), generator=g).tolist() for _ in range(B)]
            sp = SamplingParams(max_new_tokens=new_tokens, do_sample=False)
            eng.generate(prompts, sp)  # warm-up + graph capture for this bucket
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            run.prefill(torch.tensor(prompts[:1]), [0])
            torch.cuda.synchronize()
            prefill_ms = (time.perf_counter() - t0) * 1e3
            run.release(0)  # hand the slot's KV pages back before the engine admits the batch
            reqs = [eng.add_request(p, sp) for p in prompts]
            eng.step()
            torch.cuda.synchronize()
            s0, t0 = eng.stats["decode_steps"], time.perf_counter()
            eng.run_until_done(reqs)
            torch.cuda.synchronize()
            dt = time.perf_counter() - t0
            n = eng.stats["decode_steps"] - s0
            tp = emulate_tp if emu is not None else world
            out.append({"metric": f"{model_name} TP={tp} decode" + (" (rank-0 emulation, 1 GPU)" if emu else ""),
                        "batch": B, "prompt_len": prompt_len,
                        "prefill_ms": round(prefill_ms, 2), "decode_ms_per_token": round(dt / max(n, 1) * 1e3, 3),
                        "tokens_per_s": round((sum(len(r.output) for r in reqs) - 2 * B) / dt, 1),
                        "layers": cfg.n_layers, "tp": tp, "load_s": round(load_s, 1), "dtype": dtype,
                        "custom_allreduce": ar is not None, "ctrl": chan.kind if chan is not None else None,
                        "pipelined": bool(eng.pipeline),
                        "step_launches": runner.step_launches.get(next((b for b in sorted(runner.step_launches)
                                                                       if b >= B), B)),
                        "launch_structure": ("real-TP fused tails" if runner._tp_ar is not None else
                                             "single-device fused layer"),
                        "data": "random-init weights"})
            if emu is not None:
                out[-1].update(_emulation_notes(model, cfg, B, emulate_tp))
        if world > 1:
            run.shutdown()
    if ar is not None:
        ar.check()
    if world > 1:
        dist.barrier(group=ctrl)
        chan.close()
        dist.destroy_process_group(ctrl)
    del runner, model
    torch.cuda.empty_cache()
    return out


def _emulation_notes(model, cfg, B, tp):
    """What the rank-local run streams and what it leaves out (the collectives)."""
    nbytes = sum(p.numel() * p.element_size() for n, p in model.named_parameters() if n != "wte.weight")
    head = model.lm_head.local_weight()
    stream = nbytes + head.numel() * head.element_size()  # layers + LN params + the head's vocab shard
    return {"emulated_rank": 0, "rank_weight_gb": round(stream / 1e9, 2),
            "weight_floor_ms_6p3tbs": round(stream / 6.3e12 * 1e3, 2),
            "collectives_excluded": {"all_reduce_per_token": 2 * cfg.n_layers,
                                     "all_reduce_bytes": B * cfg.hidden * 2,
                                     "all_gather_logits_bytes": B * (cfg.vocab_size // tp) * 2,
                                     "note": "with the rank-local custom all-reduce the fused all-reduce tails run "
                                             "(staging, sync round, tail) with the rank as its only peer; a TP=8 "
                                             "node adds the xGMI reads of the 7 peers' partials and the "
                                             "system-scope release / acquire of each sync round (elided at "
                                             "world 1), priced by allreduce_bench"}}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="bloom-176b")
    ap.add_argument("--layers", type=int, default=0)
    ap.add_argument("--batches", default="1,8,32")
    ap.add_argument("--prompt-len", type=int, default=128)
    ap.add_argument("--new-tokens", type=int, default=64)
    ap.add_argument("--no-custom-ar", action="store_true", help="TP all-reduces through RCCL only")
    ap.add_argument("--dtype", choices=["bf16", "fp16"], default="bf16",
                    help="fp16: BASELINE config 4's dtype (native fp16 decode step)")
    ap.add_argument("--emulate-tp", type=int, default=0,
                    help="N > 1: rank 0 of a TP=N layout on this one GPU, stand-in collectives")
    ap.add_argument("--force-pg", action="store_true",
                    help="one-rank RCCL process group: TP modules + collectives captured in the decode graph")
    args = ap.parse_args()
    from kubernetes_cloud_amd.parallel.dist import init_distributed
    if not args.emulate_tp:
        init_distributed()
    if args.force_pg and not dist.is_initialized():
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29511")
        dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    recs = run_tp_decode(args.model, args.layers, [int(b) for b in args.batches.split(",")], args.prompt_len,
                         args.new_tokens, custom_ar=not args.no_custom_ar, dtype=args.dtype,
                         emulate_tp=args.emulate_tp)
    for r in recs or ():
        print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
