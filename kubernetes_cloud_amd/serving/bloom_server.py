"""bloom-inference-server compatible HTTP API (S5: the DeepSpeed-Inference BLOOM
deployment, online-inference/bloom-176b-deepspeed).

The reference image runs the external ``transformers-bloom-inference`` server
(Dockerfile:1-15) patched so that its ``generate`` returns
``GenerateResponse(text=..., num_generated_tokens=...)`` and resolves the
model from a read-only HF hub cache (files/isvc-patch.txt:18-31, 55-77). This
module serves the same routes on top of our continuous-batching engine:

* ``POST /generate/``  ``{"text": str | [str], "max_new_tokens", "min_length",
  "do_sample", "temperature", "top_k", "top_p", "repetition_penalty",
  "remove_input_from_output", ...}`` -> ``{"text": [...],
  "num_generated_tokens": [...], "query_id": n, "total_time_taken": "x secs"}``
* ``POST /tokenize/``  ``{"text": [...]}`` -> ``{"token_ids": [[...]], ...}``
* ``GET /query_id/``   -> ``{"query_id": n}``

``resolve_hf_cache_path`` is the read-only cache resolution of the patch:
``{cache}/models--{org}--{repo}/refs/{revision}`` holds the snapshot hash,
the files are under ``snapshots/{hash}``.
"""
from __future__ import annotations

import os
import threading
import time

from fastapi import Request  # module level: route annotations resolve in module globals


def resolve_hf_cache_path(model_name: str, cache_dir: str | None = None, revision: str = "main") -> str:
    """Local snapshot directory of ``org/repo`` in an HF hub cache, without
    writing to it (the PVC is mounted read-only in the InferenceService)."""
    if os.path.isdir(model_name):
        return model_name
    cache_dir = cache_dir or os.getenv("TRANSFORMERS_CACHE") or os.path.join(
        os.getenv("HF_HOME", os.path.expanduser("~/.cache/huggingface")), "hub")
    org, repo = model_name.split("/", 1)
    root = os.path.join(cache_dir, f"models--{org}--{repo}")
    ref = os.path.join(root, "refs", revision)
    if os.path.exists(ref):
        with open(ref) as f:
            sha = f.read().strip()
    else:  # a commit hash given as revision, or a single snapshot present
        snaps = os.listdir(os.path.join(root, "snapshots"))
        sha = revision if revision in snaps else sorted(snaps)[-1]
    path = os.path.join(root, "snapshots", sha)
    if not os.path.isdir(path):
        raise FileNotFoundError(path)
    return path


_GEN_KEYS = ("min_length", "do_sample", "temperature", "top_k", "top_p", "repetition_penalty",
             "max_new_tokens", "max_length", "eos_token_id", "typical_p", "num_return_sequences")


def add_routes(app, generator) -> None:
    """Register the bloom-inference-server routes on a FastAPI ``app`` served by
    ``generator`` (a ``serving.text.TextGenerator``)."""
    from fastapi.responses import JSONResponse

    state = {"query_id": 0}
    lock = threading.Lock()

    def next_id():
        with lock:
            q = state["query_id"]
            state["query_id"] += 1
            return q

    def _generate(body: dict) -> dict:
        t0 = time.perf_counter()
        texts = body.get("text")
        if isinstance(texts, str):
            texts = [texts]
        if not isinstance(texts, list) or not all(isinstance(t, str) for t in texts):
            raise ValueError("'text' must be a string or a list of strings")
        kw = {k: body[k] for k in _GEN_KEYS if body.get(k) is not None}
        kw.setdefault("max_new_tokens", 40)
        kw.pop("num_return_sequences", None)
        tok = generator.tokenizer
        enc = [tok.encode(t) for t in texts]
        params = [generator.sampling_params(len(ids), **kw) for ids in enc]
        reqs = generator.generate_ids(enc, params)
        remove = bool(body.get("remove_input_from_output", False))
        out_text, n_gen = [], []
        for t, r in zip(texts, reqs):
            new = tok.decode(r.output, skip_special_tokens=True)
            out_text.append(new if remove else t + new)
            n_gen.append(len(r.output))
        return {"text": out_text, "num_generated_tokens": n_gen, "query_id": next_id(),
                "total_time_taken": f"{time.perf_counter() - t0:.2f} secs"}

    async def generate(request: Request):
        import asyncio
        body = await request.json()
        try:
            res = await asyncio.get_running_loop().run_in_executor(None, _generate, body)
        except (ValueError, TypeError) as e:
            return JSONResponse({"error": str(e), "query_id": next_id()}, status_code=400)
        return res

    async def tokenize(request: Request):
        t0 = time.perf_counter()
        body = await request.json()
        texts = body.get("text")
        if isinstance(texts, str):
            texts = [texts]
        ids = [generator.tokenizer.encode(t) for t in texts]
        return {"token_ids": ids, "query_id": next_id(), "total_time_taken": f"{time.perf_counter() - t0:.2f} secs"}

    def query_id():
        return {"query_id": state["query_id"]}

    for path in ("/generate/", "/generate"):
        app.add_api_route(path, generate, methods=["POST"])
    for path in ("/tokenize/", "/tokenize"):
        app.add_api_route(path, tokenize, methods=["POST"])
    app.add_api_route("/query_id/", query_id, methods=["GET"])


__all__ = ["add_routes", "resolve_hf_cache_path"]
