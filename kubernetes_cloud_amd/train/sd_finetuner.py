"""Stable Diffusion finetuner / DreamBooth trainer (T8), native stack.

CLI-compatible with sd-finetuner-workflow/sd-finetuner/finetuner.py:45-258
(plain argparse, ``bool_t`` booleans, underscore flags) and the flags the
workflows render (sd-finetune-workflow-template.yaml:292-373,
db-workflow-template.yaml:257-280) -- including ``--resize``, which the
workflow passes but the reference parser rejects (accepted).

Training step (finetuner.py:467-547): frozen VAE encode -> latents * scale,
noise + random timesteps, DDPM add_noise, frozen CLIP text encoder, UNet
prediction, epsilon / v target, fp32 MSE (+ prior-preservation term for
DreamBooth), clip 1.0, AdamW, LR schedule, EMA. The UNet's parameters live in
the flat-buffer engine (bucketed all-reduce / ZeRO over RCCL across ranks);
EMA is a fused HIP lerp over the flat fp32 master (the reference's decay bug,
finetuner.py:317-334, is fixed: standard warmup EMA). Output: the diffusers
pipeline layout in ``--output_path`` every ``--save_steps`` and at the end.
"""
from __future__ import annotations

import argparse
import math
import os
import random
import sys
import time

import torch

from ..config.flags import bool_t


def build_parser() -> argparse.ArgumentParser:
    p = argparse.ArgumentParser(description="Stable Diffusion finetuner (MI355X native)")
    p.add_argument("--model", type=str, default=None)
    p.add_argument("--run_name", type=str, default=None)
    p.add_argument("--lr", type=float, default=5e-6)
    p.add_argument("--lr_scheduler", type=str, default="constant")
    p.add_argument("--lr_warmup_steps", type=int, default=0)
    p.add_argument("--epochs", type=int, default=10)
    p.add_argument("--batch_size", type=int, default=1)
    p.add_argument("--use_ema", type=bool_t, default="False")
    p.add_argument("--gradient_checkpointing", type=bool_t, default="False")
    p.add_argument("--use_8bit_adam", type=bool_t, default="False")
    p.add_argument("--adam_beta1", type=float, default=0.9)
    p.add_argument("--adam_beta2", type=float, default=0.999)
    p.add_argument("--adam_weight_decay", type=float, default=1e-2)
    p.add_argument("--adam_epsilon", type=float, default=1e-08)
    p.add_argument("--seed", type=int, default=42)
    p.add_argument("--output_path", type=str, default="./output")
    p.add_argument("--save_steps", type=int, default=500)
    p.add_argument("--resolution", type=int, default=512)
    p.add_argument("--center_crop", type=bool_t, default="True")
    p.add_argument("--resize_interp", type=str, default="lanczos")
    p.add_argument("--resize", type=bool_t, default="True", help="accepted for workflow parity (always resized)")
    p.add_argument("--shuffle", type=bool_t, default="True")
    p.add_argument("--hf_token", type=str, default=None)
    p.add_argument("--project_id", type=str, default="diffusers")
    p.add_argument("--fp16", type=bool_t, default="False")
    p.add_argument("--image_log_steps", type=int, default=10)
    p.add_argument("--image_log_amount", type=int, default=4)
    p.add_argument("--dataset", type=str, default=None)
    p.add_argument("--ucg", type=float, default=0.1)
    p.add_argument("--instance_dataset", type=str, default=None)
    p.add_argument("--instance_prompt", type=str, default=None)
    p.add_argument("--class_dataset", type=str, default=None)
    p.add_argument("--class_prompt", type=str, default=None)
    p.add_argument("--prior_loss_weight", type=float, default=1.0)
    p.add_argument("--num_class_images", type=int, default=100)
    # native extensions
    p.add_argument("--max_steps", type=int, default=-1)
    p.add_argument("--zero_stage", type=int, default=1)
    p.add_argument("--local_rank", type=int, default=-1)
    p.add_argument("--logs", type=str, default=None)
    return p


def parse_args(argv=None):
    args = build_parser().parse_args(argv)
    db = ["instance_dataset", "instance_prompt", "class_dataset", "class_prompt"]
    vals = [getattr(args, k) for k in db]
    if any(vals):
        if not all(vals):
            raise SystemExit(f"All the following values must be set when using dreambooth finetuning: {db}")
        args.is_dreambooth = True
    else:
        if not args.dataset:
            raise SystemExit("--dataset must be provided when not using dreambooth finetuning")
        args.is_dreambooth = False
    return args


def sd_lr(step: int, base: float, kind: str, warmup: int, total: int) -> float:
    """diffusers get_scheduler: constant, constant_with_warmup, linear, cosine."""
    if kind == "constant":
        return base
    if warmup and step < warmup:
        return base * step / max(1, warmup)
    if kind == "constant_with_warmup":
        return base
    prog = (step - warmup) / max(1, total - warmup)
    if kind == "cosine":
        return base * 0.5 * (1 + math.cos(math.pi * min(prog, 1.0)))
    return base * max(0.0, 1 - prog)


class FlatEMA:
    """Standard EMA with diffusers-style warmup decay min(decay, (1+t)/(10+t))
    over the engine's flat fp32 master (one fused kernel per step)."""

    def __init__(self, master: torch.Tensor, decay: float = 0.9999):
        self.shadow = master.detach().clone()
        self.decay = decay
        self.step_n = 0

    @torch.no_grad()
    def step(self, master: torch.Tensor):
        self.step_n += 1
        d = min(self.decay, (1 + self.step_n) / (10 + self.step_n))
        from ..ops import _lib
        if master.is_cuda and _lib.has("kca_ema"):
            _lib.call("kca_ema", self.shadow.data_ptr(), master.data_ptr(), float(d), master.numel(), _lib.stream())
        else:
            self.shadow.lerp_(master, 1.0 - d)


def main(argv=None):
    args = parse_args(argv)
    from ..data.images import DreamBoothDataset, LocalBase, PromptDataset
    from ..models.schedulers import DDPMScheduler, load_scheduler
    from ..models.sd_pipeline import StableDiffusionPipeline
    from ..models.vae import L_SCALE_FACTOR
    from ..obs.metrics import MetricsSink
    from ..ops import mse_loss
    from ..parallel.dist import barrier, init_distributed
    from ..utils.memory import MemoryUsage, host_info
    from .engine import TrainEngine

    info = init_distributed()
    rank, world = info.rank, info.world_size
    dev = torch.device("cuda", torch.cuda.current_device()) if torch.cuda.is_available() else torch.device("cpu")
    dtype = torch.bfloat16 if dev.type == "cuda" else torch.float32
    torch.manual_seed(args.seed + rank)
    random.seed(args.seed + rank)
    if info.is_main:
        os.makedirs(args.output_path, exist_ok=True)
        print(f"RUN_NAME: {args.run_name}\nHOST: {host_info()}\nMODEL: {args.model}\nFP16(bf16): {args.fp16}\n"
              f"RESOLUTION: {args.resolution}\nRANDOM SEED: {args.seed}", file=sys.stderr)

    pipe = StableDiffusionPipeline.from_pretrained(args.model, device=dev, dtype=dtype)
    unet, vae, te, tok = pipe.unet, pipe.vae, pipe.text_encoder, pipe.tokenizer
    vae.requires_grad_(False)
    te.requires_grad_(False)
    vae.eval()
    te.eval()
    if args.gradient_checkpointing:
        unet.enable_gradient_checkpointing()
    noise_sched = load_scheduler(os.path.join(args.model, "scheduler"), "DDPMScheduler")
    pred_type = noise_sched.prediction_type

    def gen_class_images(n: int):
        """Prior-preservation class images, data-parallel (PAR-13): prompt batch j
        runs on rank j % world (the sharding ``accelerator.prepare(sample_dataloader)``
        gives the reference, sd-finetuner/finetuner.py:612-625); each batch is
        seeded by its first index, so the images do not depend on the world
        size. Files are ``{index}-{sha1(image)}.jpg`` as in the reference."""
        import hashlib
        ds = PromptDataset(args.class_prompt, n)
        os.makedirs(args.class_dataset, exist_ok=True)
        bs = max(1, args.batch_size)
        for j, i in enumerate(range(0, n, bs)):
            if j % world != rank:
                continue
            items = [ds[k] for k in range(i, min(n, i + bs))]
            imgs = pipe([it["prompt"] for it in items], height=args.resolution, width=args.resolution,
                        num_inference_steps=int(os.environ.get("KCA_CLASS_IMAGE_STEPS", "50")),
                        generator=torch.Generator(device=dev).manual_seed(args.seed + i))
            for it, im in zip(items, imgs):
                h = hashlib.sha1(im.tobytes()).hexdigest()
                im.save(os.path.join(args.class_dataset, f"{it['index']}-{h}.jpg"))
        barrier()

    tf = dict(size=args.resolution, center_crop=args.center_crop, interpolation=args.resize_interp)
    if args.is_dreambooth:
        ds = DreamBoothDataset(tok, args.instance_dataset, args.instance_prompt, args.class_prompt,
                               args.class_dataset, args.num_class_images, gen_class_images, sync=barrier, **tf)
    else:
        ds = LocalBase(tok, args.dataset, ucg=args.ucg, shuffle=args.shuffle, **tf)
    # one sampler for every world size: the same seeded permutation, rank r taking every world-th sample,
    # so a world-W step consumes exactly the samples of a world-1 step with batch W x batch_size
    sampler = torch.utils.data.DistributedSampler(ds, world, rank, shuffle=args.shuffle, seed=args.seed)
    dl = torch.utils.data.DataLoader(ds, batch_size=args.batch_size, shuffle=False,
                                     sampler=sampler, collate_fn=ds.get_collate_fn(), num_workers=2,
                                     drop_last=world > 1)
    if args.use_8bit_adam and info.is_main:
        print("--use_8bit_adam: block-wise 8-bit AdamW states (kca_adamw8bit)", file=sys.stderr)
    unet.train()
    if next(unet.parameters()).is_cuda:
        from ..models.unet import to_channels_last
        # NHWC activations and conv weights end to end (the engine keeps the NHWC order in its flat buffer)
        to_channels_last(unet)
        to_channels_last(vae)
    eng = TrainEngine(unet, lr=args.lr, betas=(args.adam_beta1, args.adam_beta2), eps=args.adam_epsilon,
                      weight_decay=args.adam_weight_decay, max_grad_norm=1.0,
                      zero_stage=args.zero_stage if world > 1 else 0, grad_accum=1,
                      optim_bits=8 if args.use_8bit_adam else 32)
    ema = FlatEMA(eng.opt.master) if args.use_ema else None
    total = args.epochs * len(dl)
    if args.max_steps > 0:
        total = min(total, args.max_steps)
    sink = MetricsSink(args.logs or os.path.join(args.output_path, "logs"), args.run_name or "sd", args.project_id,
                       enabled=info.is_main, config={k: v for k, v in vars(args).items() if k != "hf_token"})
    scale = vae.config.scaling_factor or L_SCALE_FACTOR
    from ..ops.sd_train import mse_split, noise_prep
    fused_step = (dev.type == "cuda" and dtype == torch.bfloat16
                  and os.environ.get("KCA_SD_FUSED_TRAIN", "1") not in ("0", "false"))
    acp_dev = noise_sched.alphas_cumprod.to(dev).float()

    def save():
        if ema is not None:  # export the EMA weights, then restore the live ones
            eng.publish(ema.shadow)
        if info.is_main:
            pipe.save_pretrained(args.output_path)
        if ema is not None:
            eng.publish(eng.opt.master)
        barrier()

    step = 0
    for epoch in range(args.epochs):
        if sampler is not None:
            sampler.set_epoch(epoch)
        for batch in dl:
            if step >= total:
                break
            t0 = time.perf_counter()
            px = batch["pixel_values"].to(dev, dtype)
            ids = batch["input_ids"].to(dev)
            if fused_step:  # K18/K20 + K19: sample, noise, target and the split MSE as two fused kernels
                with torch.no_grad():
                    mean, logvar = vae.encode_moments(px).chunk(2, dim=1)
                    ctx = te(ids)
                # timesteps and noise per GLOBAL sample (rank r's sample j is sample r + W j of the step
                # under the interleaving sampler): a data-parallel step draws what one process would
                nb = mean.shape[0]
                tg = torch.Generator().manual_seed(args.seed * 7919 + step)
                ts = torch.randint(0, noise_sched.N, (nb * info.world_size,), generator=tg)
                ts = ts[info.rank::info.world_size][:nb].to(dev, non_blocking=True)
                noisy, target = noise_prep(mean, logvar, acp_dev[ts], scale, pred_type == "v_prediction",
                                           seed=args.seed * 1000003 + step, sample_base=info.rank,
                                           sample_stride=info.world_size)
                pred = unet(noisy, ts, ctx)
                loss = mse_split(pred, target, args.prior_loss_weight if args.is_dreambooth else None)
            else:
                with torch.no_grad():
                    lat = vae.encode(px).sample() * scale
                    ctx = te(ids)
                noise = torch.randn_like(lat)
                ts = torch.randint(0, noise_sched.N, (lat.shape[0],), device=dev)
                noisy = noise_sched.add_noise(lat, noise, ts)
                pred = unet(noisy, ts, ctx)
                target = noise if pred_type == "epsilon" else noise_sched.get_velocity(lat, noise, ts)
                if args.is_dreambooth:
                    p_i, p_c = pred.chunk(2)
                    t_i, t_c = target.chunk(2)
                    loss = mse_loss(p_i, t_i) + args.prior_loss_weight * mse_loss(p_c, t_c)
                else:
                    loss = mse_loss(pred, target)
            lr = sd_lr(step, args.lr, args.lr_scheduler, args.lr_warmup_steps, total)
            eng.backward(loss)
            eng.step(lr)
            if ema is not None:
                ema.step(eng.opt.master)
            step += 1
            if dev.type == "cuda":
                torch.cuda.synchronize()
            dt_s = time.perf_counter() - t0
            rsps = args.batch_size / dt_s
            lv = loss.detach().float().reshape(1)
            if world > 1:  # the step's loss over the whole (global) batch, as one process would log it
                torch.distributed.all_reduce(lv)
                lv = lv / world
            logs = {"train/loss": float(lv), "train/grad_norm": eng.grad_norm(), "train/lr": lr,
                    "train/epoch": epoch, "train/step": step,
                    "train/samples_seen": step * args.batch_size * world,
                    "perf/rank_samples_per_second": rsps, "perf/world_samples_per_second": rsps * world}
            sink.log(logs, step=step)
            if info.is_main and step % 10 == 0:
                print(f"\nLOSS: {logs['train/loss']} {MemoryUsage.now()}", file=sys.stderr, flush=True)
            if args.save_steps and step % args.save_steps == 0:
                save()
            if info.is_main and args.image_log_steps and step % args.image_log_steps == 0:
                prompt = tok.decode(ids[random.randint(0, len(ids) - 1)].tolist(), skip_special_tokens=True)
                unet.eval()
                imgs = pipe([prompt] * max(1, args.image_log_amount), height=args.resolution,
                            width=args.resolution, num_inference_steps=20)
                unet.train()
                d = os.path.join(args.output_path, "samples")
                os.makedirs(d, exist_ok=True)
                for i, im in enumerate(imgs):
                    im.save(os.path.join(d, f"step{step:06d}-{i}.png"))
        if step >= total:
            break
    barrier()
    save()
    sink.close()
    if info.is_main:
        print("Done!", file=sys.stderr)
    return {"steps": step}


if __name__ == "__main__":
    main()
