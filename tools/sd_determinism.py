"""Same-seed determinism probe for the SD serving path on the GPU: runs the
tiny test pipeline twice (fused sampler on / off) and reports where the latents
of the two calls first diverge (UNet graph replay, sampler step, VAE)."""
import os
import sys
import tempfile

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests"))


def main():
    from helpers import make_sd_dir

    from kubernetes_cloud_amd.models.sd_pipeline import StableDiffusionPipeline
    tmp = tempfile.mkdtemp()
    d = make_sd_dir(os.path.join(tmp, "sd"))
    pipe = StableDiffusionPipeline.from_pretrained(d, device="cuda", dtype=torch.bfloat16,
                                                   scheduler="LMSDiscreteScheduler")
    g = torch.Generator().manual_seed(3)
    f = 2 ** (len(pipe.vae.config.block_out_channels) - 1)
    C, L = pipe.unet.config.in_channels, 32 // f
    lat = torch.randn(1, C, L, L, generator=g)
    for fused in ("1", "0"):
        os.environ["KCA_SD_FUSED_STEP"] = fused
        outs = []
        for _ in range(3):
            x = pipe(["a fox"], height=32, width=32, num_inference_steps=4, guidance_scale=5.0, latents=lat,
                     output_type="latent")
            img = pipe(["a fox"], height=32, width=32, num_inference_steps=4, guidance_scale=5.0, latents=lat,
                       output_type="tensor")
            outs.append((x.clone(), img.clone()))
        for k in (1, 2):
            print(f"fused={fused} call0 vs call{k}: latent max diff {float((outs[0][0] - outs[k][0]).abs().max()):.3e}"
                  f" image max diff {float((outs[0][1] - outs[k][1]).abs().max()):.3e}", flush=True)
    # UNet replay alone
    run = pipe._runner()
    xin = torch.randn(2, C, L, L, device="cuda").to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    ctx = torch.cat([pipe.encode_prompt([""]), pipe.encode_prompt(["a fox"])])
    tt = torch.full((2,), 500.0, device="cuda")
    a = run(xin, tt, ctx).clone()
    b = run(xin, tt, ctx).clone()
    e = pipe.unet(xin, tt, ctx)
    print(f"unet replay vs replay {float((a - b).abs().max()):.3e}  replay vs eager "
          f"{float((a.float() - e.float()).abs().max()):.3e}", flush=True)
    z = (torch.randn(1, C, L, L, device="cuda") / pipe.scaling_factor).to(torch.bfloat16)
    v1 = pipe.vae.decode(z).float()
    v2 = pipe.vae.decode(z).float()
    print(f"vae decode twice {float((v1 - v2).abs().max()):.3e}", flush=True)
    te1 = pipe.encode_prompt(["a fox"])
    te2 = pipe.encode_prompt(["a fox"])
    print(f"text encoder twice {float((te1.float() - te2.float()).abs().max()):.3e}", flush=True)


def predictor():
    """The SDPredictor path of tests/test_entrypoints_gpu.py: tensorized load, micro-batching thread."""
    import threading

    from helpers import make_sd_dir

    from kubernetes_cloud_amd.serving.sd_service import SDPredictor, serialize_main
    tmp = tempfile.mkdtemp()
    d = make_sd_dir(os.path.join(tmp, "sd"))
    serialize_main(["--model-id", d, "--save-path", os.path.join(tmp, "tz")])
    for mb in (1, 4):
        p = SDPredictor(model_name="sd", model_id=os.path.join(tmp, "tz"), tensorized=True, num_inference_steps=4,
                        width=32, height=32, max_batch=mb, batch_window_ms=20)
        p.load()
        req = {"prompt": "a fox", "parameters": {"seed": 3, "guidance_scale": 5}}
        pngs = [p.predict(req) for _ in range(6)]
        print(f"predictor max_batch={mb}: png equal {[pngs[0] == x for x in pngs]}", flush=True)
        rp = p.configure_request(req, dict(p.parameters))
        outs = []
        for _ in range(2):
            lat = torch.cat([p._latents(rp, 3)])
            with torch.no_grad():
                outs.append(p.pipeline(["a fox"], height=32, width=32, num_inference_steps=4, guidance_scale=5.0,
                                       latents=lat, output_type="tensor").clone())
        box = []
        t = threading.Thread(target=lambda: box.append(p.pipeline(["a fox"], height=32, width=32,
                                                                  num_inference_steps=4, guidance_scale=5.0,
                                                                  latents=p._latents(rp, 3),
                                                                  output_type="tensor").clone()))
        t.start()
        t.join()
        print(f"  main-thread diff {float((outs[0] - outs[1]).abs().max()):.3e}, worker-thread vs main "
              f"{float((outs[0] - box[0]).abs().max()):.3e}", flush=True)


def modules():
    """Eager UNet + VAE + text encoder of the tensorized pipeline, repeated on fixed
    inputs: names the first module whose output changes between runs."""
    from helpers import make_sd_dir

    from kubernetes_cloud_amd.models.sd_pipeline import StableDiffusionPipeline, serialize_pipeline
    tmp = tempfile.mkdtemp()
    d = make_sd_dir(os.path.join(tmp, "sd"))
    serialize_pipeline(StableDiffusionPipeline.from_pretrained(d), os.path.join(tmp, "tz"))
    pipe = StableDiffusionPipeline.from_tensorized(os.path.join(tmp, "tz"), device="cuda", dtype=torch.bfloat16)
    f = 2 ** (len(pipe.vae.config.block_out_channels) - 1)
    C, L = pipe.unet.config.in_channels, 32 // f
    torch.manual_seed(0)
    xin = torch.randn(2, C, L, L, device="cuda").to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    tt = torch.full((2,), 500.0, device="cuda")
    z = torch.randn(1, C, L, L, device="cuda").to(torch.bfloat16)
    rec = {}
    order = []

    def hook(name):
        def fn(mod, inp, out):
            if isinstance(out, torch.Tensor):
                rec.setdefault(name, []).append(out.detach().float().clone())
                if name not in order:
                    order.append(name)
        return fn
    for root, tag in ((pipe.unet, "unet"), (pipe.vae, "vae"), (pipe.text_encoder, "te")):
        for n, m in root.named_modules():
            m.register_forward_hook(hook(f"{tag}.{n}"))
    with torch.no_grad():
        for _ in range(12):  # noqa: B007
            ctx = torch.cat([pipe.encode_prompt([""]), pipe.encode_prompt(["a fox"])])
            pipe.unet(xin, tt, ctx)
            pipe.vae.decode(z)
    per = {n: len(rec[n]) // 12 for n in order}  # calls per iteration (the text encoder runs twice)
    bad = [n for n in order if any(not torch.equal(rec[n][i % per[n]], r) for i, r in enumerate(rec[n]))]
    print(f"{len(order)} modules, {len(bad)} nondeterministic; first: {bad[:8]}", flush=True)
    for n in bad[:3]:
        diffs = [float((rec[n][i % per[n]] - r).abs().max()) for i, r in enumerate(rec[n])]
        print(f"  {n}: max diffs {diffs}", flush=True)


def steps():
    """Full tensorized pipeline calls, recording every UNet input / output: the first
    (call, step) whose output changes for an unchanged input names the UNet; a changed
    input with unchanged previous outputs names the sampler."""
    from helpers import make_sd_dir

    from kubernetes_cloud_amd.models.sd_pipeline import StableDiffusionPipeline, serialize_pipeline
    tmp = tempfile.mkdtemp()
    d = make_sd_dir(os.path.join(tmp, "sd"))
    serialize_pipeline(StableDiffusionPipeline.from_pretrained(d), os.path.join(tmp, "tz"))
    pipe = StableDiffusionPipeline.from_tensorized(os.path.join(tmp, "tz"), device="cuda", dtype=torch.bfloat16,
                                                   scheduler="LMSDiscreteScheduler")
    f = 2 ** (len(pipe.vae.config.block_out_channels) - 1)
    C, L = pipe.unet.config.in_channels, 32 // f
    lat = torch.randn(1, C, L, L, generator=torch.Generator().manual_seed(3))
    real = pipe._runner()
    log = []

    class Rec:
        unet = pipe.unet

        def __call__(self, x, t, ctx):
            if os.environ.get("PROBE_SYNC_BEFORE") == "1":
                torch.cuda.synchronize()
            out = real(x, t, ctx)
            if os.environ.get("PROBE_SYNC_AFTER") == "1":
                torch.cuda.synchronize()
            log[-1].append((x.float().clone(), ctx.float().clone(), out.float().clone()))
            return out
    rec = Rec()
    pipe._runner = lambda: rec
    res = []
    for _ in range(10):
        log.append([])
        res.append(pipe(["a fox"], height=32, width=32, num_inference_steps=4, guidance_scale=5.0, latents=lat,
                        output_type="tensor").clone())
    for c in range(1, 10):
        msg = f"call {c}: image diff {float((res[c] - res[0]).abs().max()):.3e}"
        for i, ((x0, c0, o0), (x1, c1, o1)) in enumerate(zip(log[0], log[c])):
            if not (torch.equal(x0, x1) and torch.equal(c0, c1) and torch.equal(o0, o1)):
                msg += (f"; step {i}: xin diff {float((x0 - x1).abs().max()):.2e} ctx diff "
                        f"{float((c0 - c1).abs().max()):.2e} eps diff {float((o0 - o1).abs().max()):.2e}")
                break
        print(msg, flush=True)


def graph_modules():
    """UNet module outputs inside the HIP graph: forward hooks clone every module's output,
    so the clones are captured with the graph and hold each replay's values; the replays
    at the last timestep of 10 pipeline calls are compared module by module."""
    from helpers import make_sd_dir

    from kubernetes_cloud_amd.models.sd_pipeline import StableDiffusionPipeline, serialize_pipeline
    tmp = tempfile.mkdtemp()
    d = make_sd_dir(os.path.join(tmp, "sd"))
    serialize_pipeline(StableDiffusionPipeline.from_pretrained(d), os.path.join(tmp, "tz"))
    pipe = StableDiffusionPipeline.from_tensorized(os.path.join(tmp, "tz"), device="cuda", dtype=torch.bfloat16,
                                                   scheduler="LMSDiscreteScheduler")
    f = 2 ** (len(pipe.vae.config.block_out_channels) - 1)
    C, L = pipe.unet.config.in_channels, 32 // f
    lat = torch.randn(1, C, L, L, generator=torch.Generator().manual_seed(3))
    live, order = {}, []

    def hook(name):
        def fn(mod, inp, out):
            if isinstance(out, torch.Tensor):
                live[name] = out.detach().clone()
                if name not in order:
                    order.append(name)
        return fn
    for n, m in pipe.unet.named_modules():
        m.register_forward_hook(hook(n or "unet"))
    real = pipe._runner()
    snaps, step = [], [0]

    class Rec:
        unet = pipe.unet

        def __call__(self, x, t, ctx):
            out = real(x, t, ctx)
            if step[0] % 4 == 3:
                snaps.append({n: live[n].float().cpu() for n in order})
            step[0] += 1
            return out
    rec = Rec()
    pipe._runner = lambda: rec
    for _ in range(10):
        pipe(["a fox"], height=32, width=32, num_inference_steps=4, guidance_scale=5.0, latents=lat,
             output_type="latent")
    for c in range(1, 10):
        bad = [n for n in order if not torch.equal(snaps[0][n], snaps[c][n])]
        first = f"{bad[0]} ({float((snaps[0][bad[0]] - snaps[c][bad[0]]).abs().max()):.2e})" if bad else "-"
        print(f"call {c}: {len(bad)} of {len(order)} modules differ; first {first}; next {bad[1:4]}", flush=True)


if __name__ == "__main__":
    if os.environ.get("PROBE_DET") == "1":
        torch.backends.cudnn.deterministic = True
    if "--graph-modules" in sys.argv:
        graph_modules()
    elif "--steps" in sys.argv:
        steps()
    elif "--modules" in sys.argv:
        modules()
    elif "--predictor" in sys.argv:
        predictor()
    else:
        main()
