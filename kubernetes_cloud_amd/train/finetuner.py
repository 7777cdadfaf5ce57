"""Causal-LM finetuner: the reference's ``finetuner.py`` CLI on the native stack.

Same flags, defaults, validators and outputs as
finetuner-workflow/finetuner/finetuner.py:63-273 (the Argo workflow renders
this command line at finetune-workflow.yaml:261-300), run by our launcher
instead of ``deepspeed.launcher.runner`` (one process per GPU, RCCL):

    python -m kubernetes_cloud_amd.launch --num_gpus N \
        -m kubernetes_cloud_amd.train.finetuner --run-name r --model /m --dataset d.tokens ...

Outputs (``{output-path}/results-{run-name}``): ``checkpoint-{step}`` every
``--save-steps`` optimizer steps, auto-resume from the newest one unless
``--no-resume``, ``final/`` with model + tokenizer + ``.ready.txt``.

Deliberate differences (documented in SURVEY §7.6): CPU runs are supported
(no unconditional ``torch.cuda.set_device``); the world size comes from the
launcher env; resume skips non-numeric entries; ``--fp16`` selects 16-bit
mixed precision, which on MI355X is bf16 (no loss scaling needed); the
vocabulary is only *grown* to ``len(tokenizer)`` (rounded up to 64 for
aligned LM-head/CE kernels), never shrunk.
"""
from __future__ import annotations

import copy
import json
import logging
import math
import os
import random
import sys
import time
from decimal import Decimal

import numpy as np
import torch

from ..config.flags import DashParser, FuzzyBoolAction, validation as val


def build_parser() -> DashParser:
    p = DashParser(description="Simple Text Model Finetuner")
    p.add_argument("--run-name", type=str, help="The run name to use", required=True)
    p.add_argument("--model", type=str, required=True,
                   help="The model to train against (directory, or HuggingFace ID)")
    p.add_argument("--trust-remote-code", action=FuzzyBoolAction, default=False,
                   help="Whether to trust remote code coming with the model")
    p.add_argument("--dataset", type=val.extant_file, required=True, help="Pre-tokenized dataset to use")
    p.add_argument("--tensorizer-uri", type=str, default="",
                   help="An S3 URI or path to use to load pretrained weights for Tensorizer")
    p.add_argument("--lr", type=val.non_negative(float), default=5e-5, help="Learning rate")
    p.add_argument("--epochs", type=val.positive(int), default=1, help="Number of epochs to train for")
    p.add_argument("--train-ratio", type=val.at_most_1(val.non_negative(Decimal)), default=Decimal("0.9"),
                   help="Ratio of train to value from dataset")
    p.add_argument("--warmup-ratio", type=val.at_most_1(val.non_negative(Decimal)), default=Decimal("0.1"),
                   help="Ratio of warmup steps to total steps")
    p.add_argument("--eot", type=str, default="", help="EOT token to use")
    p.add_argument("--pad", type=str, default="", help="Pad token to use")
    p.add_argument("--bs", type=val.positive(int, special_val=-1), default=-1,
                   help="Batch size (-1 == autosize)")
    p.add_argument("--bs-divisor", type=val.positive(Decimal), default=Decimal(1),
                   help="Batch size divisor for automatically determining batch size")
    p.add_argument("--gradients", type=val.positive(int), default=5, help="Gradient accumulation steps")
    p.add_argument("--zero-stage", type=int, default=3, choices=range(0, 4), help="ZeRO optimizer stage")
    p.add_argument("--seed", type=val.at_most_32_bit(val.non_negative(int)), default=42,
                   help="Random seed value")
    p.add_argument("--output-path", type=str, default="./", help="Root path of all output")
    p.add_argument("--no-resume", action=FuzzyBoolAction, dest="resume", default=True,
                   help="Do not resume from last checkpoint")
    p.add_argument("--cache", type=str, default="/tmp", help="HuggingFace cache location")
    p.add_argument("--save-steps", type=val.non_negative(int), default=500,
                   help="# of steps between checkpoint saves")
    p.add_argument("--context-size", type=val.positive(int), default=2048, help="Dataset context sizes")
    p.add_argument("--project-id", type=str, default="huggingface", help="Project ID for reporting")
    p.add_argument("--logs", type=str, default="./logs", help="Log directory location")
    p.add_argument("--ds-config", type=val.optional_extant_file, default="",
                   help="DeepSpeed configuration (zero_optimization / optimizer / clipping subset)")
    p.add_argument("--fp16", action=FuzzyBoolAction, default=False, help="Force training in fp16")
    p.add_argument("--fp16-full-eval", action=FuzzyBoolAction, default=False,
                   help="Evaluate in fp16, not in fp32 or mixed precision")
    p.add_argument("--no-shuffle", action=FuzzyBoolAction, dest="shuffle", default=True,
                   help="Disable shuffling contexts")
    p.add_argument("--prompt-file", type=val.optional_extant_file, help="Prompt file to use for checkpoint sampling")
    p.add_argument("--prompt-every", type=val.non_negative(int, special_val=-1), default=0,
                   help="Prompt every N steps")
    p.add_argument("--prompt-tokens", type=val.non_negative(int), default=200,
                   help="Number of tokens to sample from prompt")
    p.add_argument("--prompt-samples", type=val.non_negative(int), default=5, help="Number of samples to generate")
    p.add_argument("--top-k", type=val.non_negative(int), default=50, help="Top K to use for prompt sampling")
    p.add_argument("--top-p", type=val.at_most_1(val.non_negative(float)), default=0.95,
                   help="Top P to use for prompt sampling")
    p.add_argument("--temperature", type=val.positive(float), default=1.0,
                   help="Temperature to use for prompt sampling")
    p.add_argument("--repetition-penalty", type=val.positive(float), default=1.1,
                   help="Repetition penalty to use for prompt sampling")
    p.add_argument("--local-rank", type=val.non_negative(int, special_val=-1), default=-1,
                   help="For distributed training: local_rank")
    p.add_argument("--log-level", type=str.upper, default="INFO",
                   choices=("DEBUG", "INFO", "WARNING", "ERROR", "CRITICAL"), help="Log level to use")
    # native extensions (not in the reference)
    p.add_argument("--max-steps", type=int, default=-1, help="Stop after N optimizer steps (-1: full epochs)")
    p.add_argument("--gradient-checkpointing", action=FuzzyBoolAction, default=False,
                   help="Recompute activations (288 GB HBM makes it optional for <=20B models)")
    p.add_argument("--random-init", action=FuzzyBoolAction, default=False,
                   help="Allow a model dir with config.json only (random weights)")
    return p


def resolve_model_dir(model: str, cache: str | None) -> str:
    """A local directory as is; an ``org/name`` id from the HF hub cache under
    ``cache`` (``models--org--name/snapshots/<rev>``, directly or in ``hub/``),
    else unchanged (the caller's error then names it)."""
    if os.path.isdir(model) or "/" not in model or model.startswith(("/", ".")):
        return model
    from ..serving.bloom_server import resolve_hf_cache_path
    for root in ([cache, os.path.join(cache, "hub")] if cache else []) + [None]:
        try:
            return resolve_hf_cache_path(model, root)
        except (FileNotFoundError, OSError, ValueError):
            continue
    return model


def read_prompts(path: str) -> list[str]:
    """Prompt file: JSON list of strings, or one prompt per line."""
    with open(path) as f:
        text = f.read()
    try:
        data = json.loads(text)
        if isinstance(data, list):
            return [str(x) for x in data]
    except json.JSONDecodeError:
        pass
    return [ln for ln in text.splitlines() if ln.strip()]


def estimate_batch_size(model, ctx: int, divisor: Decimal, device) -> int:
    """Auto batch size (--bs -1; finetuner.py:447-466): free HBM after the
    optimizer state / estimated activation bytes per context."""
    if device.type != "cuda":
        return 1
    torch.cuda.synchronize()
    torch.cuda.empty_cache()
    free, _ = torch.cuda.mem_get_info(device)
    cfg = model.cfg
    act = ctx * cfg.hidden * cfg.n_layers * 2 * 18 + ctx * cfg.vocab_size * 2 * 2
    bs = int(free * 0.85 / (act * float(divisor)))
    return max(1, min(bs, 64))


def _setup_logging(level: str, rank: int):
    logging.basicConfig(level=getattr(logging, level), stream=sys.stderr,
                        format=f"%(asctime)s [rank{rank}] %(levelname)s %(message)s")
    return logging.getLogger("finetuner")


def main(argv=None):
    args = build_parser().parse_args(argv)
    from ..engine.generate import GenerationConfig, generate
    from ..io.checkpoint import find_last_checkpoint, load_checkpoint, save_checkpoint, write_ready
    from ..io.hf import load_pretrained, load_tokenizer, save_pretrained
    from ..models.config import LMConfig
    from ..obs.metrics import MetricsSink, StepTimer
    from ..parallel.dist import barrier, init_distributed
    from ..data.tokenized import TokenizedDataset, collate
    from ..utils.memory import MemoryUsage, host_info
    from .engine import TrainEngine
    from .optim import lr_at

    info = init_distributed()
    rank, world = info.rank, info.world_size
    log = _setup_logging(args.log_level, rank)
    main_proc = info.is_main
    dev = torch.device("cuda", torch.cuda.current_device()) if torch.cuda.is_available() else torch.device("cpu")
    if main_proc:
        log.info(f"HOST: {host_info()}")

    # --model: a directory, or an HF id resolved in the --cache hub cache (the reference passes
    # cache_dir=args.cache to from_pretrained, finetuner.py:432,795)
    args.model = resolve_model_dir(args.model, args.cache)
    if args.trust_remote_code and main_proc:
        log.info("--trust-remote-code: accepted for CLI compatibility; remote modeling code is never executed "
                 "(models run on the native kernels; unsupported model_types fail with the list of families)")
    output_dir = os.path.abspath(os.path.join(args.output_path, "results-" + args.run_name))
    last = find_last_checkpoint(output_dir) if args.resume else None
    log.info(f"LAST CHECKPOINT: {last}")

    # tokenizer (optional: config-only dirs fall back to ids from config.json)
    tokenizer = None
    try:
        tokenizer = load_tokenizer(args.model, args.eot, args.pad)
    except Exception as e:  # noqa: BLE001
        log.warning(f"no tokenizer loaded from {args.model}: {e}")
    # weights from a tensorized file/URI: explicit --tensorizer-uri, else the reference's probe of
    # the public `tensorized` bucket for this model id (finetuner.py:395-410; 5 s timeout)
    tz_uri = args.tensorizer_uri
    if not tz_uri:
        from ..io.remote import public_tensorized_uri
        tz_uri = public_tensorized_uri(args.model, fp16=args.fp16) or ""
        if tz_uri and main_proc:
            log.info(f"{args.model} is publicly tensorized: streaming {tz_uri}")
    if tz_uri and os.path.exists(os.path.join(args.model, "config.json")):
        cfg = LMConfig.from_pretrained(args.model)
    elif tz_uri:
        from ..io.tensors import metadata
        cfg = LMConfig.from_hf(metadata(tz_uri)["config"])
    else:
        cfg = LMConfig.from_pretrained(args.model)
    eos_id = tokenizer.eos_token_id if tokenizer is not None else cfg.eos_token_id
    pad_id = tokenizer.pad_token_id if tokenizer is not None else (cfg.pad_token_id if cfg.pad_token_id is not None else eos_id)

    torch.manual_seed(args.seed)
    random.seed(args.seed)
    np.random.seed(args.seed)

    dataset = TokenizedDataset(args.dataset, args.context_size, pad_id, eos_id)
    if args.train_ratio != 1:
        if main_proc:
            log.warning("Validation statistics are not implemented; setting --train-ratio to 1.0 "
                        f"(was {args.train_ratio}) to not discard training data.")
        args.train_ratio = 1
    if main_proc:
        log.info(f"DATASET: {args.dataset} {dataset.num_tokens:,} tokens, {len(dataset):,} contexts")

    dtype = torch.bfloat16 if (dev.type == "cuda") else torch.float32
    if args.fp16 and dev.type == "cuda":
        log.info("--fp16: 16-bit mixed precision runs as bf16 on MI355X")
    if tz_uri:
        from ..io.hf import load_tensorized
        model, ld = load_tensorized(tz_uri, args.model, device=dev, dtype=dtype)
        if main_proc:
            log.info(f"TENSORIZED LOAD: {tz_uri} {ld['bytes'] / 1e9:.2f} GB in {ld['seconds']:.2f}s "
                     f"({ld['gbps']:.2f} GB/s)")
    else:
        model = load_pretrained(args.model, device=dev, dtype=dtype, random_init_if_missing=args.random_init)
    if tokenizer is not None and len(tokenizer) > model.cfg.vocab_size:
        model.resize_token_embeddings((len(tokenizer) + 63) // 64 * 64)
    model.gradient_checkpointing_enable(args.gradient_checkpointing)
    model.train()
    log.info(str(MemoryUsage.now()))

    # ds_config subset
    zero_stage, betas, eps, wd, clip = args.zero_stage, (0.9, 0.999), 1e-8, 0.01, 1.0
    bucket, comm_dtype, sched_kind = int(2e8), torch.float32, "linear"
    want_offload = want_offload_param = False
    if args.ds_config:
        with open(args.ds_config) as f:
            ds = json.load(f)
        opt = (ds.get("optimizer") or {}).get("params", {})
        if isinstance(opt.get("betas"), list):
            betas = tuple(float(b) for b in opt["betas"])
        if isinstance(opt.get("eps"), (int, float)):
            eps = float(opt["eps"])
        if isinstance(opt.get("weight_decay"), (int, float)):
            wd = float(opt["weight_decay"])
        if isinstance(ds.get("gradient_clipping"), (int, float)):
            clip = float(ds["gradient_clipping"])
        zo = ds.get("zero_optimization") or {}  # its "stage" is overridden by --zero-stage (finetuner.py:915-920)
        if isinstance(zo.get("reduce_bucket_size"), (int, float)):
            bucket = int(zo["reduce_bucket_size"])
        if (ds.get("communication_data_type") or "").lower() in ("bf16", "bfloat16", "fp16"):
            comm_dtype = torch.bfloat16
        sched = ds.get("scheduler") or {}
        if sched.get("type") == "WarmupLR":
            sched_kind = "warmup"  # linear warmup then constant (ds_config.json:19-26)
        want_offload = (zo.get("offload_optimizer") or {}).get("device") == "cpu"
        want_offload_param = (zo.get("offload_param") or {}).get("device") == "cpu"
    # ds_config offload_optimizer=cpu (and offload_param=cpu with stage 3) are honoured when
    # this rank's share of params + grads + fp32 optimizer state would not fit in HBM (or when
    # forced with KCA_OFFLOAD_OPTIMIZER=1; =0 disables it): 288 GB holds every model the
    # reference finetunes on one GPU without offload.
    offload = False
    force = os.environ.get("KCA_OFFLOAD_OPTIMIZER")
    n_par = sum(p.numel() for p in model.parameters() if p.requires_grad)
    eff = zero_stage if world > 1 else 0
    need = n_par * (2 / (world if eff >= 3 else 1) + 4 / (world if eff >= 2 else 1)
                    + 12 / (world if eff >= 1 else 1))
    if force is not None:
        offload = force not in ("0", "false", "no")
    elif want_offload:
        total = torch.cuda.get_device_properties(dev).total_memory if dev.type == "cuda" else float("inf")
        offload = need > 0.85 * total
    offload_param = offload and want_offload_param and eff >= 3
    if main_proc:
        log.info("ZeRO stage %d (effective %d): %.1f GiB/rank of params+grads+optimizer state", zero_stage, eff,
                 need / 2**30)
        log.info("optimizer state: %s%s", "host (offload_optimizer=cpu, host AdamW)" if offload else "HBM",
                 "; bf16 param shard: host (offload_param=cpu)" if offload_param else "")

    engine = TrainEngine(model, lr=args.lr, betas=betas, eps=eps, weight_decay=wd, max_grad_norm=clip,
                         zero_stage=zero_stage, grad_accum=args.gradients, bucket_elems=bucket,
                         comm_dtype=comm_dtype, offload_optimizer=offload, offload_param=offload_param)
    bs = args.bs if args.bs != -1 else estimate_batch_size(model, args.context_size, args.bs_divisor, dev)
    gas = args.gradients
    per_step = bs * gas * world
    steps_per_epoch = max(1, len(dataset) // per_step)
    total_steps = steps_per_epoch * args.epochs
    if args.max_steps > 0:
        total_steps = min(total_steps, args.max_steps)
    warmup = math.ceil(float(args.warmup_ratio) * total_steps)
    if main_proc:
        log.info(f"BS: {bs} GAS: {gas} WORLD: {world} STEPS: {total_steps} WARMUP: {warmup}")

    state = {"global_step": 0, "epoch": 0, "log_history": [], "total_steps": total_steps,
             "warmup_steps": warmup, "run_name": args.run_name}
    if last is not None:
        state = load_checkpoint(last, model, engine, rank)
        log.info(f"RESUMED from {last} at step {state['global_step']}")

    sink = MetricsSink(args.logs, args.run_name, args.project_id, enabled=main_proc, config=vars(args))
    prompts = read_prompts(args.prompt_file) if args.prompt_file else []
    prompt_every = args.prompt_every
    if prompts and prompt_every == -1:
        prompt_every = args.save_steps
    if prompts and not prompt_every:
        prompt_every = args.save_steps
    sync = torch.cuda.synchronize if dev.type == "cuda" else None
    timer = StepTimer(sync)
    flops_tok = model.cfg.flops_per_token(args.context_size)

    def order(epoch):
        idx = list(range(steps_per_epoch * per_step))
        if args.shuffle:
            g = random.Random(args.seed + epoch)
            g.shuffle(idx)
        return idx

    def sample(step):
        if tokenizer is None:
            return
        with engine.gathered():  # ZeRO-3: full weights once, not per generated token
            _sample(step)

    def _sample(step):
        model.eval()
        # --fp16-full-eval: sampling in 16-bit (bf16 on MI355X -- already the GPU weights' dtype; the fp32
        # CPU path samples from a bf16 copy)
        sm = model
        if args.fp16_full_eval and next(model.parameters()).dtype == torch.float32:
            sm = copy.deepcopy(model).to(torch.bfloat16)
        _sample_prompts(step, sm)
        model.train()

    def _sample_prompts(step, sm):
        for pr in prompts:
            ids = torch.tensor([tokenizer.encode(pr)], device=dev)
            t0 = time.time()
            res = generate(sm, ids, GenerationConfig(
                max_new_tokens=args.prompt_tokens, do_sample=True, top_k=args.top_k, top_p=args.top_p,
                temperature=args.temperature, repetition_penalty=args.repetition_penalty,
                num_return_sequences=args.prompt_samples, eos_token_id=eos_id, pad_token_id=pad_id,
                bad_words_ids=[[eos_id]] if eos_id is not None else None))
            if main_proc:
                log.info(f"STEP {step} PROMPT: {pr}  INFERENCE TIME: {time.time() - t0:.2f}s")
                for s in res.sequences:
                    log.info(f"RESPONSE: {tokenizer.decode(s.tolist(), skip_special_tokens=False)}")

    step = state["global_step"]
    start_epoch = step // steps_per_epoch
    micro = 0
    from ..io.checkpoint import AsyncCheckpointWriter
    ckpt_writer = AsyncCheckpointWriter(rank)
    fault_step = int(os.environ.get("KCA_FAULT_STEP", "-1"))
    fault_ranks = {int(r) for r in os.environ.get("KCA_FAULT_RANKS", "0").split(",") if r.strip()}
    hang_step = int(os.environ.get("KCA_FAULT_HANG_STEP", "-1"))
    from ..obs.trace import trace_range
    from ..utils.watchdog import StepWatchdog
    watchdog = StepWatchdog.from_env(rank, report_dir=output_dir)
    if watchdog is not None:
        watchdog.start()
    for epoch in range(start_epoch, args.epochs):
        idx = order(epoch)
        first = (step % steps_per_epoch) if epoch == start_epoch else 0
        for s in range(first, steps_per_epoch):
            if step >= total_steps:
                break
            if fault_step >= 0 and step == fault_step and rank in fault_ranks:
                # fault injection: die hard mid-run, like a lost node. A checkpoint still
                # being written by the async writer is then incomplete and a restart skips it (correct,
                # but timing-dependent); KCA_FAULT_AFTER_CKPT=1 lets the in-flight write land first so a
                # resume test always finds it
                if os.environ.get("KCA_FAULT_AFTER_CKPT", "0") == "1":
                    ckpt_writer.wait()
                log.error(f"KCA_FAULT_STEP={fault_step}: rank {rank} exiting")
                os._exit(17)
            if hang_step >= 0 and step == hang_step and rank in fault_ranks:
                # hang injection: a rank that stops making progress (stuck
                # collective / wedged device) -- the watchdog must catch it
                log.error(f"KCA_FAULT_HANG_STEP={hang_step}: rank {rank} hanging")
                while True:
                    time.sleep(1.0)
            base = s * per_step
            lr = lr_at(step, args.lr, total_steps, warmup, sched_kind)
            timer.start()
            loss_acc = None
            for g in range(gas):
                lo = base + (g * world + rank) * bs
                batch = collate([dataset[i] for i in idx[lo:lo + bs]])
                ids = batch["input_ids"].to(dev, non_blocking=True)
                labels = batch["labels"].to(dev, non_blocking=True)
                kv = batch["kv_len"]  # host-classified mask: None / key lengths / per-key mask
                with trace_range("forward"):
                    loss = model(ids, labels=labels, kv_len=kv.to(dev, non_blocking=True) if kv is not None else None)
                with trace_range("backward"):
                    engine.backward(loss)
                d = loss.detach().float()
                loss_acc = d if loss_acc is None else loss_acc + d
                micro += 1
                if micro % (2 * gas) == 0 and main_proc:
                    print(f"\nLOSS: {d.item():.3f} {MemoryUsage.now()}", file=sys.stderr, flush=True)
            timer.gas_done()
            with trace_range("optimizer"):
                engine.step(lr)
            step += 1
            if watchdog is not None:
                watchdog.beat(step)
            perf = timer.stop(bs * gas, world, args.context_size, flops_tok)
            rec = {"loss": (loss_acc / gas).item(), "learning_rate": lr, "epoch": epoch, **perf}
            if step % 10 == 0 or step == 1:
                rec["grad_norm"] = engine.grad_norm()
                state["log_history"].append({"step": step, **rec})
            sink.log(rec, step=step)
            if prompts and prompt_every and (step % prompt_every == 0 or step == 1):
                sample(step)
            state.update(global_step=step, epoch=epoch)
            if args.save_steps and step % args.save_steps == 0:
                ck = os.path.join(output_dir, f"checkpoint-{step}")
                with engine.gathered():  # ZeRO-3: stage3_gather_16bit_weights_on_model_save
                    ckpt_writer.save(ck, model, engine, state, {k: str(v) for k, v in vars(args).items()},
                                     tokenizer, rank, world, barrier)
                if main_proc:
                    log.info(f"saved {ck}")
        if step >= total_steps:
            break

    ckpt_writer.wait(barrier)
    barrier()
    if watchdog is not None:
        watchdog.stop()
    with engine.gathered():  # every rank joins the ZeRO-3 gathers; rank 0 writes
        if main_proc:
            final = os.path.join(output_dir, "final")
            save_pretrained(model, final)
            if tokenizer is not None:
                tokenizer.save_pretrained(final)
            write_ready(final)
            log.info(f"FINAL: {final}")
    sink.close()
    barrier()
    return state


if __name__ == "__main__":
    main()
