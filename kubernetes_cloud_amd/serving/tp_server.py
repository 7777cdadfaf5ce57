"""Tensor-parallel LLM serving launcher (BLOOM-176B TP=8 class, S5).

    torchrun --nproc-per-node 8 -m kubernetes_cloud_amd.serving.tp_server \
        --model-path /mnt/pvc/bloom [--port 8080] [--random-init bloom-176b]

Every rank loads only its TP shard (``parallel.tensor_parallel.load_tp_model``,
one tensor at a time from the safetensors checkpoint, or
``parallel.ds_inference_ckpt`` for a pre-sharded DeepSpeed-Inference
checkpoint such as microsoft/bloom-deepspeed-inference-fp16 resolved from the
HF cache with ``--model-name``) into its own GPU; rank 0
runs the KServe V1 server with the BLOOM predictor contract (bloom.py env
options and request format, ``.ready.txt`` gate) and the continuous-batching
engine; ranks 1..N-1 mirror its runner calls (``engine.tp_driver``). The
reference deployed this model with DeepSpeed-Inference/MII on 8 A100s
(bloom-176b-deepspeed/02-inference-service.yaml:22,41).
"""
from __future__ import annotations

import argparse
import logging
import os

import torch
import torch.distributed as dist

log = logging.getLogger("kca.serving")


def build_tp_engine_model(args, rank, world, group):
    from ..models.config import preset
    from ..parallel.tensor_parallel import load_tp_model
    dev = torch.device("cuda", int(os.getenv("LOCAL_RANK", rank))) if torch.cuda.is_available() else \
        torch.device("cpu")
    # DS-Inference serves BLOOM in fp16 (bloom-176b-deepspeed isvc-patch): the default here too
    dtype = {"fp16": torch.float16, "bf16": torch.bfloat16}[getattr(args, "dtype", "fp16")] \
        if dev.type == "cuda" else torch.float32
    if args.random_init:
        cfg = preset(args.random_init)
        if args.layers:
            cfg.n_layers = args.layers
        return load_tp_model(cfg, rank, world, group, device=dev, dtype=dtype, random_init=True), None
    from ..io.hf import load_tokenizer
    from ..parallel.ds_inference_ckpt import is_ds_inference_dir, load_ds_inference_tp
    if is_ds_inference_dir(args.model_path):
        # pre-sharded DeepSpeed-Inference checkpoint (microsoft/bloom-deepspeed-inference-fp16):
        # each rank reads only the tp_{rank}_* files it needs, re-sharded to this world size
        model = load_ds_inference_tp(args.model_path, rank, world, group, device=dev, dtype=dtype)
    else:
        model = load_tp_model(args.model_path, rank, world, group, device=dev, dtype=dtype)
    return model, load_tokenizer(args.model_path)


def main(argv=None):
    from ..engine.runner import ModelRunner
    from ..engine.tp_driver import CollectiveRunner, follower_loop
    from ..parallel.dist import init_distributed
    ap = argparse.ArgumentParser()
    ap.add_argument("--model-path", default=os.getenv("MODEL_PATH", "/mnt/pvc/bloom"))
    ap.add_argument("--port", type=int, default=int(os.getenv("HTTP_PORT", 8080)))
    ap.add_argument("--max-batch", type=int, default=32)
    ap.add_argument("--max-len", type=int, default=2048)
    ap.add_argument("--random-init", default=None, help="preset name: random weights (benchmarks)")
    ap.add_argument("--layers", type=int, default=0)
    ap.add_argument("--dtype", choices=["fp16", "bf16"], default=os.getenv("KCA_SERVE_DTYPE", "fp16"))
    ap.add_argument("--model-name", default=os.getenv("MODEL_NAME", ""),
                    help="org/repo resolved in the read-only HF hub cache (bloom-176b-deepspeed layout)")
    args = ap.parse_args(argv)
    if args.model_name and not args.random_init:
        from .bloom_server import resolve_hf_cache_path
        args.model_path = resolve_hf_cache_path(args.model_name)
    info = init_distributed()
    rank, world = info.rank, info.world_size
    ctrl = dist.new_group(backend="gloo")
    if rank == 0 and not args.random_init:
        from .predictors import bloom_options, wait_for_ready_file
        opts, _ = bloom_options()
        wait_for_ready_file(args.model_path, opts["MODEL_DOWNLOAD_TIMEOUT"])
    dist.barrier(group=ctrl)
    model, tok = build_tp_engine_model(args, rank, world, None)
    if world > 1:  # one-shot xGMI all-reduce for the decode-size TP reductions
        from ..parallel.custom_ar import register
        register(None)
    runner = ModelRunner(model, max_slots=args.max_batch, max_len=args.max_len)
    from ..engine.ctrl_channel import open_channel
    ctrl = open_channel(ctrl)  # shared-memory ring on one node: no collective between decode steps
    if rank != 0:
        follower_loop(runner, ctrl)
        return
    from .predictors import BloomPredictor
    from .server import ModelServer
    from .text import TextGenerator
    gen = TextGenerator(model, tok, runner=CollectiveRunner(runner, ctrl))
    pred = BloomPredictor(generator=gen)
    from .bloom_server import add_routes
    try:
        # KServe V1 (bloom.py contract) and the bloom-inference-server routes
        # (/generate/, /tokenize/, /query_id/) on the same port
        ModelServer(http_port=args.port).start([pred], extra_routes=lambda app: add_routes(app, gen))
    finally:
        gen.close()
        gen.engine.runner.shutdown()


if __name__ == "__main__":
    main()
