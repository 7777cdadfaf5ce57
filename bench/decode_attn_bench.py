"""Decode attention microbenchmark: the fused RoPE + KV-append + split-K attention
launch (``ops.decode.decode_prep_attention``) plus its split combine, GPT-J
shapes (16 heads x 256, paged KV), timed as a HIP graph of back-to-back calls
so launch gaps match the decode graph. Sweeps the split-K workgroup target
(``KCA_DECODE_WGS``: fewer, longer splits vs more, shorter ones) per batch.

    python bench/decode_attn_bench.py --ctx 600 --batch 1 8 32 --wgs 256 512 1024 2048
"""
from __future__ import annotations

import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


_HEURISTIC = None


def stamps_report(B, ctx, chunk, H=16, mode="fused", paged=True):
    """One call with the kernel's diagnostic stamps on (s_memrealtime, 100 MHz): per phase,
    the median / max over workgroups of the time since the earliest workgroup start (us)."""
    from kubernetes_cloud_amd.ops import _lib
    ns = -(-ctx // chunk)
    buf = torch.zeros(B * H * ns * 8, dtype=torch.int64, device="cuda")
    _lib.call("kca_decode_set_stamps", buf.data_ptr())
    try:
        run(B, ctx, 1024, chunk=chunk, mode=mode, paged=paged, iters=1, reps=1, cold=True)
    finally:
        _lib.call("kca_decode_set_stamps", None)
    st = buf.view(-1, 8).cpu().double()
    t0 = st[:, 0].min()
    names = ["start", "len_known", "q_ready", "pages_synced", "loop_done", "merge_synced", "end"]
    rep = {"B": B, "ctx": ctx, "chunk": chunk, "wgs": st.shape[0]}
    for k, n in enumerate(names):
        col = st[:, k]
        col = col[col > 0]
        if len(col):
            rel = (col - t0) / 100.0
            rep[n] = [round(float(rel.median()), 2), round(float(rel.max()), 2)]
    return rep


def run(B, ctx, wgs, H=16, D=256, ps=16, iters=50, chunk=0, mode="fused", paged=True, reps=5, cold=False):
    from kubernetes_cloud_amd.ops import decode as dops
    dops._DECODE_WGS = wgs
    global _HEURISTIC
    _HEURISTIC = _HEURISTIC or dops.decode_chunk
    dops.decode_chunk = (lambda *a, _c=chunk: _c) if chunk else _HEURISTIC
    dev = torch.device("cuda", 0)
    pages = -(-(ctx + 1) // ps)
    kc = torch.randn(B * pages + 1, H, ps, D, device=dev).to(torch.bfloat16)
    vc = torch.randn_like(kc)
    tbl = torch.arange(B * pages, device=dev, dtype=torch.int32).view(B, pages)
    tbl = torch.cat([tbl, torch.zeros(1, pages, device=dev, dtype=torch.int32)])
    qkv = torch.randn(B, 3 * H * D, device=dev).to(torch.bfloat16)
    slots = torch.arange(B, device=dev, dtype=torch.int32)
    kv_lens = torch.full((B,), ctx, device=dev, dtype=torch.int32)
    pos = kv_lens - 1
    rot = 64
    inv = 1.0 / (10000 ** (torch.arange(0, rot, 2, device=dev).float() / rot))
    ang = torch.arange(4096, device=dev).float()[:, None] * inv[None]
    cos, sin = ang.cos().contiguous(), ang.sin().contiguous()
    out = torch.empty(B, H * D, device=dev, dtype=torch.bfloat16)
    chunk = dops.decode_chunk(B, H, ctx)
    ws = torch.zeros(max(1, dops.decode_ws_floats(B, H, H, D, ctx, chunk)), device=dev)

    if not paged:  # contiguous slots [B, H, ctx_max, D]
        kc = torch.randn(B, H, pages * ps, D, device=dev).to(torch.bfloat16)
        vc = torch.randn_like(kc)
        tbl = None

    lnx = torch.randn(1, 4096, device=dev).to(torch.bfloat16)
    lng = torch.ones(4096, device=dev, dtype=torch.bfloat16)

    def call():
        if mode == "fused":
            dops.decode_prep_attention(qkv, H, H, D, rot, True, cos, sin, pos, slots, kc, vc, kv_lens, ctx,
                                       out=out, ws=ws, block_table=tbl)
        elif mode == "ln":  # fixed-cost reference: one-workgroup decode LayerNorm of a 4096 row
            from kubernetes_cloud_amd.ops.gemv import ln_rows
            ln_rows(lnx, lng, None, 1e-5)
        else:
            dops.decode_attention(qkv, kc, vc, slots, kv_lens, H, ctx, out=out, ws=ws, chunk=chunk,
                                  block_table=tbl)
    # cold: a 512 MiB write between calls evicts L2 and the 256 MiB MALL, as the 12 GB of weights
    # streamed between two visits of a layer's KV cache do in real decoding; the flush-only graph's
    # time is subtracted
    flush = torch.empty(512 << 20, dtype=torch.uint8, device=dev) if cold else None
    iters = min(iters, 20) if cold else iters

    def graph(body):
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            for _ in range(3):
                body()
        torch.cuda.current_stream().wait_stream(s)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            for _ in range(iters):
                body()
        g.replay()
        torch.cuda.synchronize()
        return g

    def timed(g):
        t0, t1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        best = float("inf")
        for _ in range(reps):
            t0.record()
            g.replay()
            t1.record()
            torch.cuda.synchronize()
            best = min(best, t0.elapsed_time(t1) * 1000 / iters)
        return best

    if cold:
        g = graph(lambda: (flush.zero_(), call()))
        if reps <= 1:
            return None
        best = timed(g) - timed(graph(lambda: flush.zero_()))
    else:
        g = graph(call)
        if reps <= 1:
            return None
        best = timed(g)
    kv_bytes = 2 * B * ctx * H * D * 2
    return {"mode": mode, "paged": paged, "cold": cold, "B": B, "ctx": ctx, "wgs": wgs, "chunk": chunk, "nsplit": -(-ctx // chunk), "us_per_call": round(best, 2),
            "kv_GBps": round(kv_bytes / best / 1e3, 1)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ctx", type=int, nargs="+", default=[600])
    ap.add_argument("--batch", type=int, nargs="+", default=[1, 8, 32])
    ap.add_argument("--wgs", type=int, nargs="+", default=[1024])
    ap.add_argument("--chunk", type=int, nargs="+", default=[0], help="fixed split lengths (0: the heuristic)")
    ap.add_argument("--mode", nargs="+", default=["fused"], choices=["fused", "attn", "ln"],
                    help="fused: RoPE + KV append + attention in one launch; attn: attention alone")
    ap.add_argument("--layout", nargs="+", default=["paged"], choices=["paged", "contig"])
    ap.add_argument("--stamps", action="store_true", help="per-phase in-kernel timestamps instead of timing")
    ap.add_argument("--cold", action="store_true", help="evict L2 + MALL before every call (real decode)")
    a = ap.parse_args()
    from kubernetes_cloud_amd.ops import _lib
    _lib.require()
    if a.stamps:
        for ctx in a.ctx:
            for B in a.batch:
                for c in a.chunk:
                    print(json.dumps(stamps_report(B, ctx, c or 64)), flush=True)
        return
    for ctx in a.ctx:
        for B in a.batch:
            for w in a.wgs:
                for c in a.chunk:
                    for m in a.mode:
                        for lay in a.layout:
                            print(json.dumps(run(B, ctx, w, chunk=c, mode=m, paged=lay == "paged", cold=a.cold)), flush=True)


if __name__ == "__main__":
    main()
