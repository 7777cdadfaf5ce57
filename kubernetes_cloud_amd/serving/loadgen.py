"""Load generator for the inference services (S9).

Same CLI surface as online-inference/tensorizer-isvc/benchmark/load_test.py
:183-262 (``--url``, ``--flask`` | ``--kserve``, ``--async`` (default) |
``--sync``, ``--requests`` 100, ``-v``/``-q``) and the same report (throughput,
goodput when failures occur, mean latency + sample stdev, successes,
failures), plus what a serving benchmark needs on MI355X: ``--concurrency``
(bounded in-flight requests instead of all-at-once), ``--sd`` (txt2img PNG
requests), ``--triton`` (FasterTransformer V2 tensors), ``--completion``
(the finetune inference server), p50/p90/p99 latencies and ``--json``.
"""
from __future__ import annotations

import argparse
import asyncio
import json
import logging
import random
import statistics
import sys
import time
import urllib.parse

log = logging.getLogger("kca.loadgen")

PROMPTS = [
    "Once upon a time", "The MI355X has 288 GB of HBM3E and", "Kubernetes schedules pods onto nodes by",
    "In a shocking finding, scientists discovered", "The best way to fine-tune a language model is",
    "Here is a recipe for chocolate cake:", "The capital of France is", "def fibonacci(n):",
    "A haiku about GPUs:", "The three laws of robotics are", "Tensor parallelism splits each layer",
]


def build_request(kind: str, base: str, prompt: str, model: str, i: int):
    """-> (method, url, body bytes | None, headers)."""
    if kind == "flask":
        return "GET", f"{base}/predict/{urllib.parse.quote(prompt)}", None, {}
    if kind == "kserve":
        return "POST", f"{base}/v1/models/{model}:predict", json.dumps({"instances": [prompt]}).encode(), \
            {"content-type": "application/json"}
    if kind == "sd":
        return "POST", f"{base}/v1/models/{model}:predict", json.dumps(
            {"prompt": prompt, "parameters": {"seed": i}}).encode(), {"content-type": "application/json"}
    if kind == "completion":
        return "POST", f"{base}/completion", json.dumps({"prompt": prompt, "max_new_tokens": 64}).encode(), \
            {"content-type": "application/json"}
    if kind == "triton":
        import numpy as np

        from .v2 import encode_request
        ids = np.array([[ord(c) % 50000 for c in prompt]], dtype=np.int32)
        body, hdr = encode_request({"input_ids": ids, "input_lengths": np.array([[ids.shape[1]]], dtype=np.int32),
                                    "request_output_len": np.array([[64]], dtype=np.int32),
                                    "runtime_top_k": np.array([[10]], dtype=np.int32),
                                    "random_seed": np.array([[i]], dtype=np.uint64)})
        return "POST", f"{base}/v2/models/{model}/infer", body, hdr
    raise ValueError(kind)


async def run_async(reqs, concurrency: int, timeout: float):
    """-> (latencies, seconds from the first request sent to the last response): the client's import,
    construction and teardown are outside the measured window, as they are outside the server's."""
    import httpx
    sem = asyncio.Semaphore(concurrency)
    times = []
    async with httpx.AsyncClient(timeout=timeout, limits=httpx.Limits(max_connections=concurrency)) as cl:
        async def one(r):
            async with sem:
                t0 = time.perf_counter()
                try:
                    resp = await cl.request(r[0], r[1], content=r[2], headers=r[3])
                    resp.raise_for_status()
                    times.append(time.perf_counter() - t0)
                except Exception as e:  # noqa: BLE001
                    log.info("request failed: %s", e)
        t0 = time.perf_counter()
        await asyncio.gather(*(one(r) for r in reqs))
        total = time.perf_counter() - t0
    return times, total


def run_sync(reqs, timeout: float):
    import httpx
    times = []
    with httpx.Client(timeout=timeout) as cl:
        t0 = time.perf_counter()  # the whole run's window (throughput)
        for r in reqs:
            ts = time.perf_counter()  # this request's start (latency)
            try:
                resp = cl.request(r[0], r[1], content=r[2], headers=r[3])
                resp.raise_for_status()
                times.append(time.perf_counter() - ts)
            except Exception as e:  # noqa: BLE001
                log.info("request failed: %s", e)
        total = time.perf_counter() - t0
    return times, total


def _proc_worker(args):
    """One client process of ``benchmark(processes=P)``: wait for the common start time, then run its
    share -> (latencies, wall-clock first send, wall-clock last response)."""
    reqs, concurrency, timeout, start_at = args
    time.sleep(max(0.0, start_at - time.time()))
    t0 = time.time()
    times, total = asyncio.run(run_async(reqs, concurrency, timeout))
    return times, t0, t0 + total


def run_processes(reqs, concurrency: int, timeout: float, processes: int):
    """The async client split over ``processes`` processes (request i to process i % P, concurrency
    divided among them) starting at one wall-clock instant: a single asyncio + httpx process spends
    ~1-2 ms of Python per request, which at concurrency 32 is itself the bottleneck."""
    import multiprocessing as mp
    P = max(1, min(processes, concurrency))
    shares = [reqs[i::P] for i in range(P)]
    concs = [concurrency // P + (1 if i < concurrency % P else 0) for i in range(P)]
    start_at = time.time() + 3.0  # (room for the children's interpreter start and imports)
    with mp.get_context("spawn").Pool(P) as pool:
        outs = pool.map(_proc_worker, [(sh, c, timeout, start_at) for sh, c in zip(shares, concs)])
    times = [t for o in outs for t in o[0]]
    return times, max(o[2] for o in outs) - min(o[1] for o in outs)


def benchmark(url: str, kind: str, n: int, asynchronous: bool = True, concurrency: int | None = None,
              model: str = "gptj", prompts=None, timeout: float = 600.0, seed: int = 0, processes: int = 1) -> dict:
    rnd = random.Random(seed)
    prompts = prompts or PROMPTS
    reqs = [build_request(kind, url.rstrip("/"), rnd.choice(prompts), model, i) for i in range(n)]
    print("Started benchmark", flush=True)
    if asynchronous and processes > 1:
        times, total = run_processes(reqs, concurrency or n, timeout, processes)
    elif asynchronous:
        times, total = asyncio.run(run_async(reqs, concurrency or n, timeout))
    else:
        times, total = run_sync(reqs, timeout)
    ok = len(times)
    res = {"url": url, "kind": kind, "requests": n, "seconds": total, "successes": ok, "failures": n - ok,
           "throughput_rps": n / total, "goodput_rps": ok / total}
    if ok:
        st = sorted(times)
        res.update(mean_latency_s=statistics.mean(st), stdev_latency_s=statistics.stdev(st) if ok > 1 else 0.0,
                   p50_s=st[int(0.5 * (ok - 1))], p90_s=st[int(0.9 * (ok - 1))], p99_s=st[int(0.99 * (ok - 1))])
    return res


def report(r: dict):
    print(f"Benchmark finished for {r['url']} in {r['seconds']:.2f} seconds. Statistics:")
    print(f"Average throughput: {r['throughput_rps']:.4f} requests/second")
    if r["throughput_rps"] != r["goodput_rps"]:
        print(f"Average goodput: {r['goodput_rps']:.4f} successes/second")
    if "mean_latency_s" in r:
        print(f"Average latency: {r['mean_latency_s']:.4f} seconds/request"
              f" (sample standard deviation: {r['stdev_latency_s']:.4f})")
        print(f"Latency p50/p90/p99: {r['p50_s']:.4f} / {r['p90_s']:.4f} / {r['p99_s']:.4f} s")
    print(f"Successes: {r['successes']}")
    print(f"Failures: {r['failures']}")


def main(argv=None):
    p = argparse.ArgumentParser(description="Inference service load test")
    p.add_argument("--url", required=True, help="InferenceService URL")
    g = p.add_mutually_exclusive_group(required=True)
    for k in ("flask", "kserve", "sd", "triton", "completion"):
        g.add_argument(f"--{k}", dest="kind", action="store_const", const=k)
    p.set_defaults(asynchronous=True, log_level=logging.WARNING)
    s = p.add_mutually_exclusive_group()
    s.add_argument("--async", dest="asynchronous", action="store_true")
    s.add_argument("--sync", dest="asynchronous", action="store_false")
    p.add_argument("--requests", type=int, default=100)
    p.add_argument("--concurrency", type=int, default=0, help="max in-flight requests (default: all)")
    p.add_argument("--model-name", default="gptj")
    p.add_argument("--prompts-file", default="")
    p.add_argument("--json", action="store_true")
    p.add_argument("--seed", type=int, default=0, help="prompt choice seed")
    p.add_argument("--processes", type=int, default=1, help="client processes sharing the load (async mode)")
    p.add_argument("--verbose", "-v", dest="log_level", action="store_const", const=logging.INFO)
    p.add_argument("--quiet", "-q", dest="log_level", action="store_const", const=logging.ERROR)
    a = p.parse_args(argv)
    if a.requests < 1:
        p.error("--requests must be positive")
    logging.basicConfig(level=a.log_level, stream=sys.stdout)
    prompts = None
    if a.prompts_file:
        with open(a.prompts_file) as f:
            prompts = [ln.strip() for ln in f if ln.strip()]
    r = benchmark(a.url, a.kind, a.requests, a.asynchronous, a.concurrency or None, a.model_name, prompts,
                  seed=a.seed, processes=a.processes)
    print(json.dumps(r)) if a.json else report(r)
    return r


if __name__ == "__main__":
    main()
