#!/usr/bin/env python3
"""Headline benchmark: GPT-J-6B causal-LM finetune throughput (tokens/s), bf16.

Metric / config from BASELINE.json ("GPT-J-6B finetune tokens/sec ... at
1/2/4/8 MI355X"): tokens/s = world_samples_per_second x context (2048), the
reference's own formula (finetuner-workflow/finetuner/finetuner.py:516-522).
Random-init GPT-J-6B (28 x 4096, 16 heads x 256, rotary 64, vocab 50400) on
synthetic uniform token ids -- no network for checkpoints or datasets.

One timed step = one optimizer step = GAS micro-batches (forward + backward
through the native kernels) + bucketed RCCL reduce-scatter (N>1) + fused
AdamW + bf16 all-gather. Weak scaling: per-GPU work is fixed as N grows.

    python bench.py --gpus N --steps K --warmup W
    (N>1: either under `python -m torch.distributed.run --nproc-per-node N ...`,
     or plain -- without WORLD_SIZE in the env the script re-launches itself
     as N ranks, kubernetes_cloud_amd/launch.py)

Secondary measurements in the same JSON line (each bounded and fenced off, so
the headline always prints):

* ``secondary``             SD-1.5 txt2img images/s (BASELINE config 5; one
                            replica per GPU, 3 timed batches);
* ``bloom_tp``              N > 1: BLOOM-176B TP=N decode, all 70 layers
                            (BASELINE config 4);
* ``allreduce_sweep``       N > 1: custom xGMI one-/two-shot vs RCCL
                            latency by message size (bench/allreduce_bench.py);
* N = 1 only (``--extra``):
  ``secondary_dreambooth``  SD-1.5 DreamBooth samples/s (BASELINE config 3,
                            the reference formula: instance batch / step time);
  ``secondary_decode``      GPT-J-6B and GPT-NeoX-20B decode ms/token at batch 1
                            and 32, prompt 512, greedy and FT top_k 10 (the two
                            FasterTransformer serving rows);
  ``secondary_bloom_tp8_rank`` BLOOM-176B TP=8, rank 0's shard of all 70 layers +
                            its vocab shard of the head on this one GPU, stand-in
                            collectives (parallel/tp_emulation.py), batch 1/8/32;
  ``secondary_weight_load`` GPT-J fp16 and BLOOM TP=8 rank-0 shard ``.tensors``
                            -> HBM GB/s (files written in the run, O_DIRECT read)
                            next to the raw O_DIRECT storage read rate;
  ``secondary_serving``     the tensorized GPT-J KServe predictor and the BLOOM
                            predictor over HTTP (bench/serving_bench.py):
                            req/s, p50/p99, tokens/s at concurrency 1/8/32, and
                            the same requests without the HTTP layer.

``KCA_BENCH_SHARED_GPU=1`` (rehearsal only, parallel/shared_gpu.py): N ranks
share cuda:0 with gloo collectives staged through the host, so the N > 1 paths
run on a one-GPU box; pair it with ``--layers/--hidden`` shrink flags, which
make the number a rehearsal, not a measurement (flagged in ``config``).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--model", default="gpt-j-6b")
    # micro-batch 16 x GAS 2 (global 32): the largest micro-batch that fits 288 GB
    # (peak 216 GiB), as the reference's auto batch size picks the largest that fits
    # (finetuner.py:447-466); vs 8 x 4: 32.7k -> 33.5k tok/s (profiles/bench_gptj_r1_v13_mb16.log)
    ap.add_argument("--micro-batch", type=int, default=16)
    ap.add_argument("--gas", type=int, default=2)
    ap.add_argument("--seq", type=int, default=2048)
    ap.add_argument("--zero-stage", type=int, default=1)
    ap.add_argument("--ckpt", action="store_true", help="activation checkpointing")
    ap.add_argument("--bucket", type=float, default=2e8)
    ap.add_argument("--profile-steps", type=int, default=0)
    ap.add_argument("--tunableop", choices=["auto", "use", "tune", "off"], default="auto",
                    help="hipBLASLt/rocBLAS solution selection via PyTorch TunableOp: 'tune' measures during "
                         "warmup and writes tuning/tunableop_results.csv; 'auto' uses that file when present")
    ap.add_argument("--tunableop-file", default=os.path.join(ROOT, "tuning", "tunableop_results.csv"))
    ap.add_argument("--sd", type=int, default=1, help="also measure the SD-1.5 txt2img half of the BASELINE metric "
                    "(batch 8, 512 px, 50 LMS steps, CFG 7; one rank-local replica per GPU) after the GPT-J steps")
    ap.add_argument("--bloom-tp", choices=["auto", "on", "off"], default="auto",
                    help="also measure BLOOM-176B TP=N decode (BASELINE config 4) after the GPT-J steps; "
                         "'auto' = when N > 1")
    ap.add_argument("--bloom-layers", type=int, default=0, help="0 = all 70 layers")
    ap.add_argument("--bloom-timeout", type=float, default=420.0,
                    help="seconds; if the BLOOM phase overruns, the headline line is printed without it")
    ap.add_argument("--bloom-batches", default="1,8,32")
    ap.add_argument("--extra", choices=["auto", "on", "off"], default="auto",
                    help="N=1 secondaries (DreamBooth, GPT-J decode, BLOOM 8-layer slice, weight load); "
                         "'auto' = when N == 1")
    ap.add_argument("--extra-timeout", type=float, default=600.0,
                    help="seconds for all N=1 secondaries together; on overrun the line prints with what finished")
    # rehearsal shrink flags (tests/test_bench_shared_gpu.py): NOT the BASELINE config
    ap.add_argument("--layers", type=int, default=0)
    ap.add_argument("--hidden", type=int, default=0)
    ap.add_argument("--heads", type=int, default=0)
    args = ap.parse_args()

    # `python bench.py --gpus N` outside torchrun: re-run this script as N ranks
    # (torchrun's env contract) before anything touches the GPU, and exit with
    # their status. Under torchrun WORLD_SIZE is set and this is skipped.
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        from kubernetes_cloud_amd.launch import self_launch_argv, spawn
        cmds, envs = self_launch_argv(os.path.abspath(__file__), sys.argv[1:], args.gpus)
        sys.exit(spawn(cmds, envs))
    if os.environ.get("KCA_BENCH_DRYRUN") == "1":  # CPU test of the launch contract (tests/test_launch_cpu.py)
        print(f"[bench] dryrun rank {os.environ.get('RANK', '0')} "
              + json.dumps({"world_size": int(os.environ.get("WORLD_SIZE", "1"))}), flush=True)
        return

    import torch
    import torch.distributed as dist
    from kubernetes_cloud_amd.models.causal_lm import build_model
    from kubernetes_cloud_amd.models.config import preset
    from kubernetes_cloud_amd.parallel.dist import init_distributed
    from kubernetes_cloud_amd.train.engine import TrainEngine
    from kubernetes_cloud_amd.ops import _lib

    from kubernetes_cloud_amd.parallel import shared_gpu
    shared = shared_gpu.enabled()
    if shared:  # rehearsal: every rank on cuda:0, gloo collectives staged through the host
        torch.cuda.set_device(0)
        info = init_distributed(backend="gloo")
        shared_gpu.install()
    else:
        info = init_distributed()
    world = info.world_size
    if world != args.gpus and info.is_main:
        print(f"[bench] note: --gpus {args.gpus} but WORLD_SIZE={world}; reporting the real world size",
              file=sys.stderr)
    if torch.cuda.device_count() < world and not shared:
        raise SystemExit(f"[bench] {world} ranks but only {torch.cuda.device_count()} visible GPUs")
    dev = torch.device("cuda", torch.cuda.current_device())
    _lib.require()
    torch.manual_seed(1234 + info.rank)

    tfile = args.tunableop_file
    mode = args.tunableop
    if mode == "auto":
        mode = "use" if os.path.exists(tfile) else "off"
    if args.tunableop == "off":
        os.environ["KCA_TUNABLEOP"] = "off"
    if mode != "off":
        import torch.cuda.tunable as tunable
        os.makedirs(os.path.dirname(tfile), exist_ok=True)
        tunable.enable(True)
        tunable.set_filename(tfile, insert_device_ordinal=False)
        tunable.tuning_enable(mode == "tune")
        if mode == "use":
            tunable.read_file(tfile)
        if mode == "tune":
            tunable.set_max_tuning_duration(40)

    shrink = {k: v for k, v in (("n_layer", args.layers), ("n_embd", args.hidden), ("n_head", args.heads)) if v}
    cfg = preset(args.model, **shrink)
    model = build_model(cfg, device=dev, dtype=torch.bfloat16, seed=0)
    model.gradient_checkpointing_enable(args.ckpt)
    model.train()
    eng = TrainEngine(model, lr=5e-5, betas=(0.9, 0.999), eps=1e-8, weight_decay=0.01,
                      max_grad_norm=1.0, zero_stage=args.zero_stage, grad_accum=args.gas,
                      bucket_elems=int(args.bucket))
    B, S = args.micro_batch, args.seq
    gen = torch.Generator(device=dev)
    gen.manual_seed(17 + info.rank)
    batches = [torch.randint(0, cfg.vocab_size, (B, S), device=dev, generator=gen)
               for _ in range(args.gas)]

    def loss_fn(ids):
        return model(ids, labels=ids)

    def one_step():
        return eng.train_batch(batches, loss_fn, lr=5e-5)

    for i in range(args.warmup):
        loss = one_step()
    if mode == "tune":  # results are written to the file at interpreter exit
        torch.cuda.synchronize()
        tunable.tuning_enable(False)
        if info.is_main:
            print(f"[bench] warmup {i} loss={loss.item():.4f} mem={torch.cuda.max_memory_allocated()/2**30:.1f}GiB",
                  file=sys.stderr, flush=True)
    if dist.is_initialized():
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(args.steps):
        loss = one_step()
    if dist.is_initialized():
        dist.barrier()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    if dist.is_initialized():
        t = torch.tensor([dt], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
    global_batch = B * args.gas * world
    peak_gib = torch.cuda.max_memory_allocated() / 2**30
    tokens = args.steps * global_batch * S
    tps = tokens / dt
    ms = dt / args.steps * 1e3
    flops_tok = cfg.flops_per_token(S)
    mfu = tps * flops_tok / (world * 2.5e15)
    loss_v = float(loss.item())
    eng.remove_hooks()  # drops the gradient-sink references to the engine
    del eng, model, batches
    torch.cuda.empty_cache()
    rec = None
    if info.is_main:
        print(f"[bench] loss={loss_v:.4f} step={ms:.1f}ms tokens/s={tps:.0f} "
              f"tokens/s/gpu={tps/world:.0f} MFU(2.5PF dense)={mfu*100:.1f}% "
              f"peak_mem={peak_gib:.1f}GiB", file=sys.stderr, flush=True)
        rec = {
            "metric": "GPT-J-6B finetune tokens/sec",
            "value": round(tps, 1),
            "unit": "tokens/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms, 2),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "bf16",
            "data": "synthetic (uniform random token ids; random-init weights)",
            "config": {
                "model": args.model,
                "global_batch": global_batch,
                "micro_batch": B,
                "grad_accum": args.gas,
                "seq_len": S,
                "parallelism": f"dp{world}" + (f"-zero{args.zero_stage}" if world > 1 else ""),
                "activation_checkpointing": bool(args.ckpt),
                "mfu_2p5pf": round(mfu, 4),
                "peak_mem_gib": round(peak_gib, 1),
            },
            "secondary": None,
        }
        if shrink or shared:  # rehearsal runs are never a BASELINE measurement
            rec["config"]["rehearsal"] = {"shrink": shrink, "shared_gpu": shared}
    if args.sd:
        sd = _sd_txt2img(dev, world, info.is_main)
        if rec is not None:
            rec["secondary"] = sd
    if args.bloom_tp == "on" or (args.bloom_tp == "auto" and world > 1):
        bloom = _bloom_tp(args, info, rec)
        if rec is not None:
            rec["bloom_tp"] = bloom
    if args.extra == "on" or (args.extra == "auto" and world == 1):
        _extras(args, dev, rec)
    if rec is not None:
        summ = _summary(rec)
        rec["summary"] = summ  # last key: the tail of the (long) line carries every headline value
        print(json.dumps(rec), flush=True)
        print("[bench] summary " + json.dumps(summ, separators=(",", ":")), file=sys.stderr, flush=True)
    if dist.is_initialized():
        dist.destroy_process_group()


def _summary(rec) -> dict:
    """Every secondary's headline value in a few hundred bytes (the driver keeps
    only the tail of the ~10 KB line): txt2img, DreamBooth, decode ms/token per (model, batch,
    sampling), BLOOM TP=8 rank ms/token per batch, weight-load GB/s (and of its storage ceiling)."""
    out = {"gptj_train_tok_s": rec.get("value")}

    def val(key):
        v = rec.get(key)
        return v.get("value") if isinstance(v, dict) else None

    out["txt2img_img_s"] = val("secondary")
    out["dreambooth_samples_s"] = val("secondary_dreambooth")
    dec = rec.get("secondary_decode")
    for r in (dec or {}).get("records", []) if isinstance(dec, dict) else []:
        m = "gptj" if "gpt-j" in str(r.get("metric")) else "neox"
        s_ = "" if r.get("sampling") in (None, "greedy") else "_" + str(r["sampling"])
        s_ += "_fp16" if r.get("dtype") == "fp16" else ""
        out[f"decode_{m}_b{r.get('batch')}{s_}_ms"] = r.get("decode_ms_per_token")
    bl = rec.get("secondary_bloom_tp8_rank")
    for r in (bl or {}).get("records", []) if isinstance(bl, dict) else []:
        if isinstance(r, dict) and "batch" in r:
            f16 = "_fp16" if r.get("dtype") == "fp16" else ""
            out[f"bloom_tp8_rank_b{r['batch']}{f16}_ms"] = r.get("decode_ms_per_token")
    wl = rec.get("secondary_weight_load")
    for r in (wl or {}).get("records", []) if isinstance(wl, dict) else []:
        if isinstance(r, dict) and "gbps" in r:
            k = "bloom_shard" if "bloom" in str(r.get("model")) else "gptj"
            out[f"load_{k}_gbps"] = r.get("gbps")
            out[f"load_{k}_of_storage"] = r.get("of_storage")
            out[f"load_{k}_path"] = r.get("read_path")
    bt = rec.get("bloom_tp")
    if isinstance(bt, dict):
        for r in bt.get("records", []) or []:
            if isinstance(r, dict) and "batch" in r:
                out[f"bloom_tp{rec.get('n_gpus')}_b{r['batch']}_ms"] = r.get("decode_ms_per_token")
    return {k: v for k, v in out.items() if v is not None}


def _bloom_tp(args, info, rec):
    """BLOOM-176B TP=N decode (BASELINE config 4: prefill ms, decode ms/token,
    tokens/s at batch 1/8/32; bench/bloom_tp_bench.py) on the same ranks. A
    watchdog bounds the phase: on overrun rank 0 prints the headline record
    (marked) and every rank exits, so a stuck TP phase can never cost the
    GPT-J number."""
    import importlib.util
    import threading

    def _overrun():
        if rec is not None:
            rec["bloom_tp"] = {"error": f"timeout after {args.bloom_timeout:.0f}s"}
            print(json.dumps(rec), flush=True)
        sys.stdout.flush()
        sys.stderr.flush()
        # exit 0 on every rank, deliberately: rank 0's record above is complete and carries
        # bloom_tp.error, and a non-zero rank exit makes torch.distributed.run fail the whole job,
        # which would discard the measured GPT-J number along with the hung secondary
        os._exit(0)

    timer = threading.Timer(args.bloom_timeout, _overrun)
    timer.daemon = True
    timer.start()
    try:
        spec = importlib.util.spec_from_file_location("kca_bloom_bench", os.path.join(ROOT, "bench", "bloom_tp_bench.py"))
        mod = importlib.util.module_from_spec(spec)
        spec.loader.exec_module(mod)
        out = mod.run_tp_decode("bloom-176b", layers=args.bloom_layers,
                                batches=tuple(int(b) for b in args.bloom_batches.split(",")), prompt_len=128,
                                new_tokens=32)
        try:  # custom one-/two-shot vs RCCL by message size, on the same ranks (placing the switch points)
            sweep = _load_bench("allreduce_bench").run_sweep()
            if rec is not None:
                rec["allreduce_sweep"] = sweep
        except Exception as e:  # noqa: BLE001
            if rec is not None:
                rec["allreduce_sweep"] = {"error": repr(e)[:300]}
        return out
    except Exception as e:  # noqa: BLE001 - the headline line must still print
        if info.is_main:
            print(f"[bench] BLOOM TP measurement failed: {e!r}", file=sys.stderr, flush=True)
        return {"error": repr(e)[:300]}
    finally:
        timer.cancel()


def _sd_txt2img(dev, world, is_main):
    """SD-1.5 txt2img images/s (BASELINE.json metric, second half; BASELINE.md
    protocol: batch 8, 512x512, 50 steps, CFG 7.0, incl. VAE decode, excl. PNG
    encode), random-init weights, one replica per rank (weak scaling): total
    images / max-over-ranks mean time of three timed batches after one warmup."""
    import importlib.util

    import torch
    import torch.distributed as dist
    spec = importlib.util.spec_from_file_location("kca_sd_bench", os.path.join(ROOT, "bench", "sd_bench.py"))
    sdb = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(sdb)
    a = argparse.Namespace(batch=8, res=512, steps=3, warmup=1, infer_steps=50, scheduler="LMSDiscreteScheduler",
                           ckpt=False)
    try:
        # hipBLASLt solution choices tuned for the SD GEMM shapes (utils/tunable.py;
        # txt2img 5.55 -> 5.65 images/s in an interleaved same-box A/B)
        from kubernetes_cloud_amd.utils import tunable
        tunable.ensure(tunable.SD_FILE)
        if dist.is_initialized():
            dist.barrier()
        r = sdb.bench_infer(a, dev)
        dt = torch.tensor([r["ms_per_batch"]], dtype=torch.float64, device=dev)
        if dist.is_initialized():
            dist.all_reduce(dt, op=dist.ReduceOp.MAX)
        ms = float(dt.item())
        return {"metric": "SD-1.5 txt2img images/sec", "value": round(world * a.batch / (ms / 1e3), 3),
                "unit": "images/s", "ms_per_batch": round(ms, 1), "n_gpus": world,
                "config": dict(r["config"], replicas=world)}
    except Exception as e:  # noqa: BLE001 - the headline line must still print
        if is_main:
            print(f"[bench] SD txt2img measurement failed: {e!r}", file=sys.stderr, flush=True)
        return None


def _load_bench(name):
    import importlib.util
    spec = importlib.util.spec_from_file_location(f"kca_{name}", os.path.join(ROOT, "bench", f"{name}.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def _extras(args, dev, rec):
    """N = 1 secondaries: the BASELINE configs a one-GPU run can measure besides
    the headline and txt2img. Each is fenced (an exception records ``error``);
    a watchdog bounds them all, printing the line with what finished."""
    import threading

    import torch
    deadline = time.perf_counter() + args.extra_timeout

    def _overrun():
        if rec is not None:
            rec["extra_error"] = f"N=1 secondaries overran {args.extra_timeout:.0f}s; unfinished ones omitted"
            print(json.dumps(rec), flush=True)
        sys.stdout.flush()
        sys.stderr.flush()
        os._exit(0)

    timer = threading.Timer(args.extra_timeout, _overrun)
    timer.daemon = True
    timer.start()

    def fenced(key, fn):
        if time.perf_counter() > deadline:
            return
        t0 = time.perf_counter()
        torch.cuda.reset_peak_memory_stats()  # per-phase peaks, not the GPT-J step's
        try:
            out = fn()
        except Exception as e:  # noqa: BLE001 - the headline line must still print
            print(f"[bench] {key} failed: {e!r}", file=sys.stderr, flush=True)
            out = {"error": repr(e)[:300]}
        peak = round(torch.cuda.max_memory_allocated() / 2**30, 1)
        if isinstance(out, dict):
            out.setdefault("phase_peak_mem_gib", peak)
        elif isinstance(out, list):
            out = {"phase_peak_mem_gib": peak, "records": out}
        torch.cuda.empty_cache()
        print(f"[bench] {key}: {time.perf_counter() - t0:.1f}s", file=sys.stderr, flush=True)
        if rec is not None:
            rec[key] = out

    def dreambooth():
        sdb = _load_bench("sd_bench")
        a = argparse.Namespace(batch=8, res=512, steps=5, warmup=2, ckpt=False)
        return sdb.bench_train(a, dev)

    def decode():
        db = _load_bench("decode_bench")
        out = db.run_decode("gpt-j-6b", batches=(1, 32), prompt_len=512, new_tokens=64,
                            sampling=("greedy", "ft_topk10"))
        torch.cuda.empty_cache()
        out += db.run_decode("gpt-neox-20b", batches=(1, 32), prompt_len=512, new_tokens=64,
                             sampling=("greedy", "ft_topk10"))
        torch.cuda.empty_cache()
        # FT's data_type: fp16 (download-weights-job-gptj.yml:225-227): the native fp16 decode step
        for model in ("gpt-j-6b", "gpt-neox-20b"):
            out += db.run_decode(model, batches=(1, 32), prompt_len=512, new_tokens=64, sampling=("greedy",),
                                 dtype="fp16")
            torch.cuda.empty_cache()
        return out

    def bloom_tp8_rank():
        tb = _load_bench("bloom_tp_bench")
        recs = tb.run_tp_decode("bloom-176b", layers=0, batches=(1, 8, 32), prompt_len=128, new_tokens=32,
                                emulate_tp=8)
        torch.cuda.empty_cache()
        # DS-Inference's fp16 (bloom-176b-deepspeed isvc-patch): the native fp16 step
        recs += tb.run_tp_decode("bloom-176b", layers=0, batches=(1, 8, 32), prompt_len=128, new_tokens=32,
                                 emulate_tp=8, dtype="fp16")
        return {"layout": "rank 0 of TP=8 on one GPU: all 70 layers at the per-rank shard shapes (QKV "
                          "14336->5376, out 1792->14336, fc_in 14336->7168, fc_out 7168->14336) + the "
                          "31,360-row head shard; the all-reduces run the deployment's fused tail kernels "
                          "over a rank-local custom all-reduce (no peer traffic), the logits all-gather is a "
                          "stand-in; bf16 and fp16 records",
                "records": recs}

    def weight_load():
        d = os.environ.get("KCA_WEIGHT_LOAD_DIR", os.environ.get("TMPDIR", "/tmp"))
        wl = _load_bench("weight_load_bench")
        out = wl.run_weight_load("gpt-j-6b", d, threads=8, sources=("cold",))
        torch.cuda.empty_cache()
        # BASELINE.md:55's "one BLOOM TP shard": rank 0 of TP=8, 10 of 70 layers + the embedding,
        # extrapolated to the whole shard at the measured rate
        return out + wl.run_weight_load("bloom-176b", d, threads=8, sources=("cold",), tp=8, layers=10)

    def serving():
        # the tensorized GPT-J KServe predictor and the BLOOM predictor contract over HTTP
        # (loadgen at concurrency 1 / 8 / 32) next to the same requests straight into predict
        sb = _load_bench("serving_bench")
        d = os.environ.get("KCA_WEIGHT_LOAD_DIR", os.environ.get("TMPDIR", "/tmp"))
        out = {"gptj": sb.run_gptj(d), "bloom_slice": sb.run_bloom_slice(8)}
        torch.cuda.empty_cache()
        out["sd_txt2img"] = sb.run_sd()  # the txt2img InferenceService contract (PNG per request)
        return out

    try:
        fenced("secondary_dreambooth", dreambooth)
        fenced("secondary_decode", decode)
        fenced("secondary_bloom_tp8_rank", bloom_tp8_rank)
        fenced("secondary_weight_load", weight_load)
        fenced("secondary_serving", serving)
    finally:
        timer.cancel()


if __name__ == "__main__":
    main()
