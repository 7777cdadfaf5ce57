#!/usr/bin/env python3
"""SD-1.5 benchmarks (BASELINE.json configs 3 and 5) on random-init weights.

  --mode train : DreamBooth UNet finetune step (instance + class batch, frozen
                 VAE encode + CLIP encode, UNet fwd/bwd, prior-preservation MSE,
                 fused AdamW) -> samples/s by the reference's
                 perf/world_samples_per_second definition (sd-finetuner/
                 finetuner.py:563-568: ``args.batch_size / step_time``, where
                 batch_size counts INSTANCE examples -- each carries its class
                 image, datasets.py:122-140); images/s incl. class is reported
                 alongside
  --mode infer : txt2img batch 8, 512x512, 50 steps, CFG 7.0, incl. VAE decode,
                 excl. PNG encode -> images/s
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch

from kubernetes_cloud_amd.utils import miopen as _miopen  # noqa: E402

_miopen.configure()


def build(dev, dtype):
    from kubernetes_cloud_amd.models.clip_text import CLIPTextConfig, build_clip_text
    from kubernetes_cloud_amd.models.unet import UNetConfig, build_unet
    from kubernetes_cloud_amd.models.vae import VAEConfig, build_vae
    from kubernetes_cloud_amd.models.unet import to_channels_last
    unet = build_unet(UNetConfig(), device=dev, dtype=dtype)
    vae = build_vae(VAEConfig(), device=dev, dtype=dtype)
    te = build_clip_text(CLIPTextConfig(), device=dev, dtype=dtype)
    if os.environ.get("KCA_SD_CHANNELS_LAST", "1") not in ("0", "false"):
        to_channels_last(unet)
        to_channels_last(vae)
    return unet, vae, te


def _attrib(step):
    """--attrib: where the eager PyTorch (at::native) kernels and device copies of one step come from.
    One step under a TorchDispatchMode records the first repo stack frame of every aten call by (op,
    shapes) (the profiler's own Python stacks are empty on this build); one step under torch.profiler
    times the kernels each (op, shapes) launched. stderr."""
    import collections
    import traceback

    from torch.profiler import ProfilerActivity, profile
    from torch.utils._python_dispatch import TorchDispatchMode

    frames = collections.defaultdict(collections.Counter)

    def _shape(a):
        return list(a.shape) if isinstance(a, torch.Tensor) else []

    class _Where(TorchDispatchMode):
        def __torch_dispatch__(self, func, types, args=(), kwargs=None):
            st = traceback.extract_stack()
            fr = next((f"{f.filename.split('kubernetes_cloud_amd/')[-1]}:{f.lineno}" for f in reversed(st)
                       if "kubernetes_cloud_amd" in f.filename and "_python_dispatch" not in f.filename), "?")
            name = "aten::" + func.__name__.split(".")[0]
            frames[(name, str([_shape(x) for x in args[:2]]))][fr] += 1
            return func(*args, **(kwargs or {}))

    with _Where():
        step()
    torch.cuda.synchronize()
    with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], record_shapes=True) as prof:
        step()
        torch.cuda.synchronize()
    agg, total, eager = collections.defaultdict(lambda: [0, 0.0]), 0.0, 0.0
    for ev in prof.events():
        for k in getattr(ev, "kernels", []) or []:
            us = k.duration
            total += us
            if "at::native" not in k.name and "rocclr" not in k.name:
                continue
            eager += us
            e = ev
            while getattr(e, "cpu_parent", None) is not None and not e.name.startswith("aten::"):
                e = e.cpu_parent
            key = (e.name, str([list(x) if isinstance(x, (list, tuple)) else [] for x in e.input_shapes[:2]]))
            agg[key][0] += 1
            agg[key][1] += us
    print(f"[sd_bench attrib] kernel time {total / 1e3:.1f} ms, eager/copy {eager / 1e3:.2f} ms "
          f"({100 * eager / max(total, 1):.2f} %)", file=sys.stderr)
    for (name, shp), (n, us) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:40]:
        fr = frames.get((name, shp))
        where = ", ".join(f"{f} x{c}" for f, c in fr.most_common(2)) if fr else "?"
        print(f"  {us:9.1f} us {n:4d}x {name:22s} {shp:60s} {where}", file=sys.stderr)


def bench_train(args, dev):
    from kubernetes_cloud_amd.models.schedulers import DDPMScheduler, sd_scheduler_config
    from kubernetes_cloud_amd.ops import mse_loss
    from kubernetes_cloud_amd.train.engine import TrainEngine
    unet, vae, te = build(dev, torch.bfloat16)
    vae.requires_grad_(False)
    te.requires_grad_(False)
    if args.ckpt:
        unet.enable_gradient_checkpointing()
    unet.train()
    eng = TrainEngine(unet, lr=5e-6, weight_decay=1e-2, max_grad_norm=1.0, zero_stage=0)
    sch = DDPMScheduler.from_config(sd_scheduler_config())
    B = args.batch  # instance images per step; class images double it
    px = torch.randn(2 * B, 3, args.res, args.res, device=dev, dtype=torch.bfloat16)
    ids = torch.randint(0, 49408, (2 * B, 77), device=dev)

    from kubernetes_cloud_amd.ops.sd_train import mse_split, noise_prep
    fused = os.environ.get("KCA_SD_FUSED_TRAIN", "1") not in ("0", "false")
    acp = sch.alphas_cumprod.to(dev).float()
    it = [0]

    def step():
        t = torch.randint(0, 1000, (px.shape[0],), device=dev)
        if fused:  # the trainer's fused path (train/sd_finetuner.py): 2 kernels for sample/noise/target/MSE
            with torch.no_grad():
                mean, logvar = vae.encode_moments(px).chunk(2, dim=1)
                ctx = te(ids)
            noisy, target = noise_prep(mean, logvar, acp[t], 0.18215, False, seed=it[0])
            it[0] += 1
            loss = mse_split(unet(noisy, t, ctx), target, 1.0)
        else:
            with torch.no_grad():
                lat = vae.encode(px).sample() * 0.18215
                ctx = te(ids)
            noise = torch.randn_like(lat)
            pred = unet(sch.add_noise(lat, noise, t), t, ctx)
            pi, pc = pred.chunk(2)
            ni, nc = noise.chunk(2)
            loss = mse_loss(pi, ni) + mse_loss(pc, nc)
        eng.backward(loss)
        eng.step(5e-6)
        return loss

    for i in range(args.warmup):
        tw = time.perf_counter()
        step()
        torch.cuda.synchronize()
        print(f"[sd_bench] train warmup {i}: {time.perf_counter() - tw:.1f}s", file=sys.stderr, flush=True)
    torch.cuda.synchronize()
    if getattr(args, "attrib", False):
        _attrib(step)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        loss = step()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    sps = args.steps * B / dt  # reference formula: instance batch_size / step time
    return {"metric": "SD-1.5 DreamBooth UNet finetune samples/sec", "value": round(sps, 2),
            "unit": "samples/s", "images_per_s_incl_class": round(2 * sps, 2),
            "ms_per_step": round(dt / args.steps * 1e3, 2), "loss": float(loss.item()),
            "config": {"instance_batch": B, "class_batch": B, "resolution": args.res, "dtype": "bf16",
                       "grad_ckpt": args.ckpt, "peak_mem_gib": round(torch.cuda.max_memory_allocated() / 2**30, 1)}}


def bench_infer(args, dev):
    from kubernetes_cloud_amd.models.schedulers import load_scheduler, sd_scheduler_config
    unet, vae, te = build(dev, torch.bfloat16)
    for m in (unet, vae, te):
        m.eval()
    sch = load_scheduler(sd_scheduler_config(), args.scheduler)
    B, steps, g = args.batch, args.infer_steps, 7.0
    ids = torch.randint(0, 49408, (2 * B, 77), device=dev)
    from kubernetes_cloud_amd.models.sd_pipeline import unet_runner
    run_unet = unet_runner(unet)

    @torch.no_grad()
    def run():
        ctx = te(ids)
        sch.set_timesteps(steps, device=dev)
        x = torch.randn(B, 4, args.res // 8, args.res // 8, device=dev) * sch.init_noise_sigma
        for t in sch.timesteps:
            xin = sch.scale_model_input(torch.cat([x, x]), t).to(torch.bfloat16)
            eps = run_unet(xin, torch.full((2 * B,), float(t), device=dev), ctx).float()
            eu, ec = eps.chunk(2)
            x = sch.step(eu + g * (ec - eu), t, x).float()
        return vae.decode((x / 0.18215).to(torch.bfloat16))

    for i in range(args.warmup):
        tw = time.perf_counter()
        run()
        torch.cuda.synchronize()
        print(f"[sd_bench] infer warmup {i}: {time.perf_counter() - tw:.1f}s", file=sys.stderr, flush=True)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        img = run()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    ips = args.steps * B / dt
    return {"metric": "SD-1.5 txt2img images/sec", "value": round(ips, 3), "unit": "images/s",
            "ms_per_batch": round(dt / args.steps * 1e3, 1),
            "config": {"batch": B, "resolution": args.res, "steps": steps, "cfg": g, "scheduler": args.scheduler,
                       "dtype": "bf16", "out_shape": list(img.shape),
                       "hip_graph": type(run_unet).__name__ == "UNetGraph"}}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--mode", choices=["train", "infer", "both"], default="both")
    ap.add_argument("--batch", type=int, default=8)
    ap.add_argument("--res", type=int, default=512)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--infer-steps", type=int, default=50)
    ap.add_argument("--scheduler", default="LMSDiscreteScheduler")
    ap.add_argument("--ckpt", action="store_true")
    ap.add_argument("--deterministic", action="store_true",
                    help="MIOpen deterministic convolution solvers only (the SD predictor's setting)")
    ap.add_argument("--tunableop", choices=["auto", "use", "tune", "off"], default="auto",
                    help="hipBLASLt solution choices from tuning/tunableop_sd.csv (utils/tunable.py)")
    ap.add_argument("--tunableop-file", default=None)
    ap.add_argument("--attrib", action="store_true", help="train: attribute eager kernels of one step (stderr)")
    args = ap.parse_args()
    if args.deterministic:
        torch.backends.cudnn.deterministic = True
    dev = torch.device("cuda", 0)
    from kubernetes_cloud_amd.ops import _lib
    from kubernetes_cloud_amd.utils import tunable
    _lib.require()
    if args.tunableop == "off":
        os.environ["KCA_TUNABLEOP"] = "off"  # also keeps models/unet.py:to_channels_last from enabling it
    tmode = tunable.configure(args.tunableop_file or tunable.SD_FILE, args.tunableop)
    print(f"[sd_bench] tunableop: {tmode}", file=sys.stderr, flush=True)
    if args.mode in ("train", "both"):
        print(json.dumps(bench_train(args, dev)), flush=True)
        torch.cuda.empty_cache()
    if args.mode in ("infer", "both"):
        a2 = argparse.Namespace(**vars(args))
        a2.steps, a2.warmup = max(1, args.steps // 2), 1
        print(json.dumps(bench_infer(a2, dev)), flush=True)


if __name__ == "__main__":
    main()
