#!/usr/bin/env python3
"""Weight-load benchmark (BASELINE.md "Weight load": GB/s and seconds to ready,
PVC -> HBM for GPT-J fp16 ~12.1 GB; the reference prints the same numbers from
tensorizer at tensorizer-isvc/tensorizer_hf_isvc/load_model.py:63-73).

    python bench/weight_load_bench.py [--model gpt-j-6b] [--dir /tmp] [--http]

Writes a random-init GPT-J-6B as fp16 ``.tensors`` (config embedded), then
measures ``load_tensorized`` -- no-init model construction + native stream
into preallocated HBM parameters -- from:

* the file with O_DIRECT (storage -> pinned ring -> hipMemcpyAsync; the page
  cache is bypassed, so this is a cold read of the device),
* the same file again (steady state),
* ``--http``: a local HTTP/1.1 Range server (sendfile) through the ranged-GET
  streamer (16 keep-alive connections) -- the s3:// / https:// code path.

One JSON line per source. Random weights (no checkpoints offline).
"""
from __future__ import annotations

import argparse
import http.server
import json
import os
import sys
import threading
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch


class _SendfileRange(http.server.BaseHTTPRequestHandler):
    protocol_version = "HTTP/1.1"
    root = "/tmp"

    def log_message(self, *a):
        pass

    def do_GET(self):
        path = os.path.join(self.root, self.path.lstrip("/"))
        size = os.path.getsize(path)
        a, b = 0, size - 1
        rng = self.headers.get("Range")
        if rng:
            a, b = (int(x) for x in rng.split("=")[1].split("-"))
            b = min(b, size - 1)
        n = b - a + 1
        self.send_response(206 if rng else 200)
        self.send_header("Content-Length", str(n))
        if rng:
            self.send_header("Content-Range", f"bytes {a}-{b}/{size}")
        self.end_headers()
        self.wfile.flush()
        with open(path, "rb") as f:
            off = a
            while off <= b:
                sent = os.sendfile(self.connection.fileno(), f.fileno(), off, b + 1 - off)
                if sent <= 0:
                    break
                off += sent


def _build(cfg, dev, tp):
    if tp:  # rank 0's shard, random-init on the device (a 176B shard never touches host memory)
        from kubernetes_cloud_amd.parallel.tensor_parallel import load_tp_model
        return load_tp_model(cfg, 0, tp, None, device=dev, dtype=torch.float16, random_init=True)
    from kubernetes_cloud_amd.models.causal_lm import build_model
    return build_model(cfg, device=dev, dtype=torch.float16, seed=0)


def _load(cfg, uri, dev, tp, threads):
    """-> (model, stream stats): no-init construction + native stream into preallocated HBM."""
    from kubernetes_cloud_amd.io.hf import load_tensorized
    if not tp:
        return load_tensorized(uri, None, device=dev, dtype=torch.float16, threads=threads)
    from kubernetes_cloud_amd.io.tensors import load_into_module
    from kubernetes_cloud_amd.models.causal_lm import CausalLM
    from kubernetes_cloud_amd.parallel.tensor_parallel import tp_convert_
    with torch.device("meta"):
        model = CausalLM(cfg)
    tp_convert_(model, 0, tp, None)
    model = model.to(torch.float16).to_empty(device=dev)
    return model, load_into_module(model, uri, device=dev, threads=threads)


def run_weight_load(model="gpt-j-6b", directory="/tmp", threads=8, sources=("cold", "repeat"), tp=0, layers=0):
    """bench.py's ``secondary_weight_load``: write a random-init fp16 model (or rank 0's TP=``tp``
    shard; ``layers`` > 0: the first layers only, the record extrapolates the full shard) as
    ``.tensors`` and flush it; time no-init construction + native O_DIRECT stream into HBM FIRST (the
    file has not been read since it was written: "cold"), then price the storage with a raw O_DIRECT
    read of a separate copy. Each record carries the bytes the streamer read with O_DIRECT and the
    bytes that fell back to buffered reads. Returns one record per source; the files are removed."""
    from kubernetes_cloud_amd.io.hf import serialize_causal_lm
    from kubernetes_cloud_amd.io.native import storage_ceiling
    from kubernetes_cloud_amd.models.config import preset
    dev = torch.device("cuda", torch.cuda.current_device())
    cfg = preset(model)
    full_layers = cfg.n_layers
    if layers:
        cfg.n_layers = layers
    path = os.path.join(directory, f"kca_bench_{model}{f'_tp{tp}r0' if tp else ''}_{os.getpid()}.tensors")
    ceil_path = path + ".ceiling"
    m = _build(cfg, dev, tp)
    ref = {k: v.float().abs().sum().item() for k, v in list(m.state_dict().items())[:3]}
    layer_bytes = sum(p.numel() * p.element_size() for p in m.h[0].parameters())
    total = sum(p.numel() * p.element_size() for p in m.parameters())
    serialize_causal_lm(m, path)
    # the ceiling's copy is serialized from the model too (never read from the file the loads read)
    serialize_causal_lm(m, ceil_path)
    # flush the freshly written files before any timed read: an O_DIRECT read of a file with dirty pages
    # first writes them back (round 4's 6.75 -> 6.11 GB/s "drop")
    for p_ in (path, ceil_path):
        fd = os.open(p_, os.O_RDONLY)
        try:
            os.fsync(fd)
        finally:
            os.close(fd)
    del m
    torch.cuda.empty_cache()
    out = []
    try:
        # the storage rate of these boxes moves between reads (a ceiling read only after the loads came
        # out 10 % under the cold load on one box, profiles/bench_r6_final3.json): the separate copy is
        # priced before AND after the loads, the ceiling is the better of the two
        raw_before = storage_ceiling(ceil_path, repeats=1)
        for src in sources:
            torch.cuda.synchronize()
            t = time.perf_counter()
            model_, st = _load(cfg, path, dev, tp, threads)
            torch.cuda.synchronize()
            ready = time.perf_counter() - t
            got = {k: v.float().abs().sum().item() for k, v in list(model_.state_dict().items())[:3]}
            assert all(abs(got[k] - ref[k]) <= 1e-3 * max(1.0, ref[k]) for k in ref), (got, ref)
            rec = {"metric": "weight load", "source": f"file O_DIRECT ({src})",
                   "model": model + (f" TP={tp} rank-0 shard" if tp else ""), "dtype": "fp16",
                   "bytes": int(st["bytes"]), "gbps": round(st["gbps"], 2), "seconds_to_ready": round(ready, 3),
                   "odirect_bytes": st.get("odirect_bytes"), "buffered_bytes": st.get("buffered_bytes"),
                   "read_path": ("O_DIRECT" if not st.get("buffered_bytes") else
                                 ("buffered" if not st.get("odirect_bytes") else "mixed")),
                   "threads": threads, "data": "random-init weights"}
            if layers and layers < full_layers:  # the whole shard at the measured rate
                full = total + (full_layers - layers) * layer_bytes
                rec.update(layers=f"{layers} of {full_layers}", full_bytes=int(full),
                           full_seconds_at_rate=round(full / (st["gbps"] * 1e9), 2))
            out.append(rec)
            del model_
            torch.cuda.empty_cache()
        raw = storage_ceiling(ceil_path)  # O_DIRECT, best of several queue depths
        if raw_before["gbps"] > raw["gbps"]:
            raw = raw_before
        for rec in out:
            rec.update(storage_gbps=round(raw["gbps"], 2),
                       storage_file="separate copy (serialized, never copied from the loaded file), "
                                    "best of reads before and after the loads",
                       storage_queue=f"{raw['threads']} threads x {raw['chunk'] >> 20} MiB",
                       of_storage=round(rec["gbps"] / max(raw["gbps"], 1e-9), 3))
    finally:
        for p_ in (path, ceil_path):
            if os.path.exists(p_):
                os.remove(p_)
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="gpt-j-6b")
    ap.add_argument("--dir", default=os.environ.get("TMPDIR", "/tmp"))
    ap.add_argument("--http", action="store_true")
    ap.add_argument("--threads", type=int, default=8)
    ap.add_argument("--keep", action="store_true")
    ap.add_argument("--tp", type=int, default=0,
                    help="time rank 0's tensor-parallel shard of --model at this TP degree (BLOOM TP shard load)")
    args = ap.parse_args()
    from kubernetes_cloud_amd.io.hf import load_tensorized, serialize_causal_lm
    from kubernetes_cloud_amd.models.causal_lm import build_model
    from kubernetes_cloud_amd.models.config import preset
    dev = torch.device("cuda", 0)
    cfg = preset(args.model)
    path = os.path.join(args.dir, f"kca_{args.model}{f'_tp{args.tp}r0' if args.tp else ''}.tensors")
    t0 = time.perf_counter()
    if args.tp:  # rank 0's shard, random-init on the device (a 176B shard never touches host memory)
        from kubernetes_cloud_amd.parallel.tensor_parallel import load_tp_model
        m = load_tp_model(cfg, 0, args.tp, None, device=dev, dtype=torch.float16, random_init=True)
    else:
        m = build_model(cfg, device=dev, dtype=torch.float16, seed=0)
    ref = {k: v.float().abs().sum().item() for k, v in list(m.state_dict().items())[:3]}
    info = serialize_causal_lm(m, path)
    del m
    torch.cuda.empty_cache()
    print(f"[weight-load] wrote {info['bytes'] / 1e9:.2f} GB to {path} in {time.perf_counter() - t0:.1f}s",
          file=sys.stderr, flush=True)
    results = []

    def run(label, uri, **kw):
        torch.cuda.synchronize()
        t = time.perf_counter()
        if args.tp:
            from kubernetes_cloud_amd.io.tensors import load_into_module
            from kubernetes_cloud_amd.models.causal_lm import CausalLM
            from kubernetes_cloud_amd.parallel.tensor_parallel import tp_convert_
            with torch.device("meta"):
                model = CausalLM(cfg)
            tp_convert_(model, 0, args.tp, None)
            model = model.to(torch.float16).to_empty(device=dev)
            st = load_into_module(model, uri, device=dev, threads=args.threads)
        else:
            model, st = load_tensorized(uri, None, device=dev, dtype=torch.float16, threads=args.threads)
        torch.cuda.synchronize()
        ready = time.perf_counter() - t
        got = {k: v.float().abs().sum().item() for k, v in list(model.state_dict().items())[:3]}
        assert all(abs(got[k] - ref[k]) <= 1e-3 * max(1.0, ref[k]) for k in ref), (got, ref)
        rec = {"metric": "weight load", "source": label, "model": args.model + (f" TP={args.tp} rank-0 shard" if args.tp else ""),
               "dtype": "fp16",
               "bytes": int(st["bytes"]), "stream_s": round(st["seconds"], 3), "gbps": round(st["gbps"], 2),
               "seconds_to_ready": round(ready, 3), "threads": args.threads, "data": "random-init weights", **kw}
        print(json.dumps(rec), flush=True)
        results.append(rec)
        del model
        torch.cuda.empty_cache()

    run("file O_DIRECT (cold device read)", path)
    run("file O_DIRECT (repeat)", path)
    if args.http:
        class H(_SendfileRange):
            root = args.dir
        srv = http.server.ThreadingHTTPServer(("127.0.0.1", 0), H)
        threading.Thread(target=srv.serve_forever, daemon=True).start()
        url = f"http://127.0.0.1:{srv.server_address[1]}/{os.path.basename(path)}"
        run("http://localhost ranged GET (page-cache warm server)", url)
        srv.shutdown()
    if not args.keep:
        os.remove(path)


if __name__ == "__main__":
    main()
