#!/usr/bin/env python3
"""Same-box A/B of the fused batch-1 decode layer's launch structure.

    python bench/decode_chain_ab.py --model gpt-j-6b
    python bench/decode_chain_ab.py --model bloom-176b --emulate-tp 8

Arms (runner attributes, engine/runner.py ``_chain`` / ``_attn_out_fused``):
  chain   -- each layer's closing tail launch also streams the projection that consumes its LayerNorm
             (next QKV / LM head; BLOOM: the out-projection tail runs fc_in), ops/decode.py gemv_ln_gemv
  attn    -- BLOOM's attention + out-projection + ln_2 in one launch (decode_attn_out_ln)
One engine per model; each arm re-captures the decode graph and times pure decode steps (batch 1,
prompt 512), arms interleaved over ``--rounds`` passes. One JSON line per arm.
"""
from __future__ import annotations

import argparse
import json
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="gpt-j-6b")
    ap.add_argument("--emulate-tp", type=int, default=0)
    ap.add_argument("--layers", type=int, default=0)
    ap.add_argument("--prompt-len", type=int, default=512)
    ap.add_argument("--steps", type=int, default=48)
    ap.add_argument("--rounds", type=int, default=3)
    args = ap.parse_args()
    from kubernetes_cloud_amd.engine.llm_engine import LLMEngine, SamplingParams
    from kubernetes_cloud_amd.models.config import preset
    from kubernetes_cloud_amd.ops import _lib
    _lib.require()
    dev = torch.device("cuda", 0)
    cfg = preset(args.model)
    if args.layers:
        cfg.n_layers = args.layers
    if args.emulate_tp > 1:
        from kubernetes_cloud_amd.parallel.tp_emulation import emulated_rank_model
        m = emulated_rank_model(cfg, args.emulate_tp, 0, device=dev, dtype=torch.bfloat16)
    else:
        from kubernetes_cloud_amd.models.causal_lm import build_model
        m = build_model(cfg, device=dev, dtype=torch.bfloat16, seed=0)
    m.eval()
    total = args.rounds * 4 * (args.steps + 4) + 64
    eng = LLMEngine(m, max_slots=1, max_len=args.prompt_len + total)
    run = eng.runner
    seq = run._layer_kind == "seq"
    arms = [(1, 1), (0, 1)] + ([(1, 0), (0, 0)] if seq else [])
    g = torch.Generator().manual_seed(0)
    prompt = torch.randint(0, cfg.vocab_size, (args.prompt_len,), generator=g).tolist()
    req = eng.add_request(prompt, SamplingParams(max_new_tokens=total, do_sample=False))
    eng.step()
    times = {a: [] for a in arms}
    for _ in range(args.rounds):
        for a in arms:
            run._chain, run._attn_out_fused = bool(a[0]), bool(a[1])
            torch.cuda.synchronize()
            run._graphs.clear()  # re-capture with this arm's launch structure
            for _ in range(4):
                eng.step()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(args.steps):
                eng.step()
            torch.cuda.synchronize()
            times[a].append((time.perf_counter() - t0) / args.steps * 1e3)
            assert not req.done
    for a in arms:
        ts = times[a]
        print(json.dumps({"metric": f"{args.model} B=1 decode" + (f" TP={args.emulate_tp} rank" if args.emulate_tp else ""),
                          "chain": a[0], "attn_out_fused": a[1] if seq else None,
                          "ms_per_step_mean": round(statistics.mean(ts), 4),
                          "ms_per_step_min": round(min(ts), 4), "passes": [round(t, 4) for t in ts],
                          "layers": cfg.n_layers, "kind": run._layer_kind}), flush=True)


if __name__ == "__main__":
    main()
