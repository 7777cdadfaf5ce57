"""In-kernel timestamps of the fused B=1 decode layer kernel (decode_attn_gemv_kernel) inside a
real GPT-J decode step: the attention workgroups' phases (start, length known, Q ready, pages
staged, loop done, partials merged, end, after the split fan-in) and the fc_in GEMV workgroups'
start / end, all relative to the earliest workgroup start of the launch (s_memrealtime, 100 MHz).
Every layer's launch rewrites the same entries, so the report is the last layer of the last step.
Eager launches (no graphs: the stamp buffer is a launch argument).

    python bench/decode_layer_stamps.py --steps 8
"""
from __future__ import annotations

import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="gpt-j-6b")
    ap.add_argument("--prompt-len", type=int, default=512)
    ap.add_argument("--steps", type=int, default=8)
    args = ap.parse_args()
    from kubernetes_cloud_amd.engine.llm_engine import LLMEngine, SamplingParams
    from kubernetes_cloud_amd.models.causal_lm import build_model
    from kubernetes_cloud_amd.models.config import preset
    from kubernetes_cloud_amd.ops import _lib
    _lib.require()
    dev = torch.device("cuda", 0)
    cfg = preset(args.model)
    m = build_model(cfg, device=dev, dtype=torch.bfloat16, seed=0)
    eng = LLMEngine(m, max_slots=1, max_len=args.prompt_len + args.steps + 32, use_graphs=False)
    g = torch.Generator().manual_seed(0)
    prompt = torch.randint(0, cfg.vocab_size, (args.prompt_len,), generator=g).tolist()
    eng.add_request(prompt, SamplingParams(max_new_tokens=args.steps + 16, do_sample=False))
    for _ in range(3):
        eng.step()
    torch.cuda.synchronize()
    nwg = 8192  # >= the fused launch's grid (attention splits + fc_in row groups)
    buf = torch.zeros(nwg * 8, dtype=torch.int64, device=dev)
    _lib.call("kca_decode_set_stamps", buf.data_ptr())
    try:
        for _ in range(args.steps):
            eng.step()
        torch.cuda.synchronize()
    finally:
        _lib.call("kca_decode_set_stamps", None)
    st = buf.view(nwg, 8).cpu().double()
    used = st[:, 7] > 0
    st = st[used]
    t0 = st[:, 0][st[:, 0] > 0].min()
    attn = st[:, 1] > 0
    rel = (st - t0) / 100.0
    names = ["start", "len_known", "q_ready", "pages_synced", "loop_done", "merge_synced", "end", "after_fanin"]
    rep = {"attn_wgs": int(attn.sum()), "gemv_wgs": int((~attn).sum())}
    for k, n in enumerate(names):
        col = rel[attn, k]
        col = col[st[attn, k] > 0]
        if len(col):
            rep["attn_" + n] = [round(float(col.min()), 2), round(float(col.median()), 2), round(float(col.max()), 2)]
    for k, n in ((0, "start"), (7, "end")):
        col = rel[~attn, k]
        rep["gemv_" + n] = [round(float(col.min()), 2), round(float(col.median()), 2),
                            round(float(torch.quantile(col, 0.9)), 2), round(float(col.max()), 2)]
    rep["note"] = "[min, median, max] us since the first workgroup start (gemv: [min, median, p90, max])"
    print(json.dumps(rep), flush=True)


if __name__ == "__main__":
    main()
