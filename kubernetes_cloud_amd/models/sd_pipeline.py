"""Stable Diffusion txt2img pipeline + diffusers-layout I/O (S1/S2/T8 support).

Loads the layouts the reference produces and serves:
* a diffusers directory (``model_index.json`` + ``unet/ vae/ text_encoder/
  tokenizer/ scheduler/``) -- what the SD finetuner saves
  (sd-finetuner/finetuner.py:413-434) and the predictor loads
  (stable-diffusion/service/service.py:163-171);
* the tensorized layout (``{encoder,vae,unet}.tensors`` + ``*-config.json`` +
  tokenizer/scheduler; serializer/serialize.py:35-50, service.py:173-198).

Batched, classifier-free-guided denoise loop: one UNet call on the
[uncond; cond] 2B batch per step, guidance combine and sampler update in fp32,
VAE decode at the end. BASELINE config 5 runs it at batch 8, 512x512, 50
steps, CFG 7.0 (the reference serves batch 1 with containerConcurrency 1).
"""
from __future__ import annotations

import json
import os

import torch

from .clip_text import CLIPTextConfig, CLIPTextModel
from .schedulers import load_scheduler, sd_scheduler_config
from .unet import UNet2DConditionModel, UNetConfig, to_channels_last
from .vae import L_SCALE_FACTOR, AutoencoderKL, VAEConfig


def _read_cfg(path):
    with open(path) as f:
        return json.load(f)


def _load_module(cls, cfg, weights_dir, device, dtype, names=("diffusion_pytorch_model", "model")):
    from safetensors.torch import load_file
    with torch.device("meta"):
        m = cls(cfg)
    m = m.to_empty(device=device).to(dtype)
    sd = None
    for n in names:
        p = os.path.join(weights_dir, n + ".safetensors")
        if os.path.exists(p):
            sd = load_file(p)
            break
        p = os.path.join(weights_dir, n + ".bin")
        if os.path.exists(p):
            sd = torch.load(p, map_location="cpu", weights_only=True)
            break
    if sd is None:
        raise FileNotFoundError(f"no weights in {weights_dir}")
    if isinstance(m, CLIPTextModel):
        m.load_hf(sd)
    else:
        m.load_state_dict({k: v.to(dtype) for k, v in _map_legacy_vae(sd).items()}, strict=True)
    return m


def _map_legacy_vae(sd: dict) -> dict:
    """Older diffusers VAE checkpoints name the mid attention query/key/value/
    proj_attn; map them to to_q/to_k/to_v/to_out.0 (and squeeze 1x1 conv kernels)."""
    ren = {"query": "to_q", "key": "to_k", "value": "to_v", "proj_attn": "to_out.0"}
    out = {}
    for k, v in sd.items():
        parts = k.split(".")
        if "attentions" in parts and parts[-2] in ren:
            k = ".".join(parts[:-2] + [ren[parts[-2]], parts[-1]])
            if v.dim() == 4:
                v = v[:, :, 0, 0]
        out[k] = v
    return out


class UNetGraph:
    """The UNet denoising forward replayed as a HIP graph (one per input
    shape): SD-1.5 at 512 px is ~1000 kernel launches per step, and the host
    cannot issue them as fast as MI355X retires them at batch 8 + CFG. Inputs
    are copied into the graph's static buffers; the returned tensor is the
    graph's static output (consume it before the next call). Capture failures
    fall back to eager for that shape. ``KCA_SD_GRAPH=0`` disables."""

    def __init__(self, unet):
        self.unet = unet
        self.graphs: dict = {}
        self.pad_gen = -1
        # the text context of the last call and its cross-attention K/V: one prompt batch calls the
        # UNet with the same ``ctx`` tensor every step, so K/V are projected once per batch
        # (models/unet.py CtxKV); the strong reference keeps the address from being reused
        self._ctx_ref = None
        self._ctx_ver = -1
        self._kv_fresh = False
        self.ctx_kv = os.environ.get("KCA_SD_CTX_KV", "1") not in ("0", "false") and hasattr(unet, "ctx_kv")

    def __call__(self, x, t, ctx):
        from .unet import pad_generation
        if self.graphs and pad_generation() != self.pad_gen:
            self.graphs.clear()  # padded attention weights were rebuilt: the graphs hold stale copies
        key = (tuple(x.shape), x.dtype, tuple(t.shape), tuple(ctx.shape), ctx.dtype)
        g = self.graphs.get(key)
        if g is None:
            self._ctx_ref = None
            g = self.graphs[key] = self._capture(x, t, ctx)
        if g is False:
            return self.unet(x, t, ctx)
        graph, sx, st, sc, out = g
        sx.copy_(x)
        st.copy_(t)
        if self.ctx_kv:
            if not (ctx is self._ctx_ref and ctx._version == self._ctx_ver):
                self.unet.ctx_kv(ctx, out=sc)  # eager, once per prompt batch, into the graph's table
                self._ctx_ref, self._ctx_ver = ctx, ctx._version
        else:
            sc.copy_(ctx)
        graph.replay()
        return out

    @torch.no_grad()
    def _capture(self, x, t, ctx):
        sx, st = x.clone(), t.clone()
        sc = self.unet.ctx_kv(ctx.clone()) if self.ctx_kv else ctx.clone()
        try:
            side = torch.cuda.Stream()
            side.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(side):  # warm up: solver search, workspaces, allocator
                for _ in range(2):
                    self.unet(sx, st, sc)
            torch.cuda.current_stream().wait_stream(side)
            graph = torch.cuda.CUDAGraph()
            with torch.cuda.graph(graph, capture_error_mode="thread_local"):  # see engine/runner.py _capture
                out = self.unet(sx, st, sc)
            from .unet import pad_generation
            self.pad_gen = pad_generation()
            return graph, sx, st, sc, out
        except Exception as e:  # noqa: BLE001 - eager is always correct
            import sys
            print(f"[sd] HIP graph capture failed ({e!r}); running the UNet eagerly", file=sys.stderr)
            torch.cuda.synchronize()
            return False


def unet_runner(unet):
    """Graph-replaying runner on the GPU (eval only), the module itself otherwise."""
    if (next(unet.parameters()).is_cuda and not unet.training
            and os.environ.get("KCA_SD_GRAPH", "1") not in ("0", "false")):
        return UNetGraph(unet)
    return unet


class StableDiffusionPipeline:
    def __init__(self, unet: UNet2DConditionModel, vae: AutoencoderKL, text_encoder: CLIPTextModel,
                 tokenizer, scheduler, scaling_factor: float = L_SCALE_FACTOR):
        self.unet, self.vae, self.text_encoder = unet, vae, text_encoder
        self.tokenizer, self.scheduler = tokenizer, scheduler
        self.scaling_factor = scaling_factor
        self._layout()

    def _runner(self):
        r = getattr(self, "_unet_runner", None)
        if r is None or getattr(r, "unet", r) is not self.unet or self.unet.training:
            r = self._unet_runner = unet_runner(self.unet)
        return r

    def _layout(self):
        """On the GPU the UNet and VAE run channels-last end to end (NHWC MIOpen
        convolutions + NHWC GroupNorm kernels; models/unet.py:to_channels_last)."""
        if next(self.unet.parameters()).is_cuda:
            to_channels_last(self.unet)
            to_channels_last(self.vae)

    @property
    def device(self):
        return next(self.unet.parameters()).device

    @property
    def dtype(self):
        return next(self.unet.parameters()).dtype

    def to(self, device=None, dtype=None):
        for m in (self.unet, self.vae, self.text_encoder):
            m.to(device=device, dtype=dtype)
        self._layout()
        return self

    # ------------------------------------------------------------------ I/O
    @classmethod
    def from_pretrained(cls, path: str, device="cpu", dtype=torch.float32, scheduler: str | None = None):
        from transformers import AutoTokenizer
        unet = _load_module(UNet2DConditionModel, UNetConfig.from_pretrained(os.path.join(path, "unet")),
                            os.path.join(path, "unet"), device, dtype)
        vae = _load_module(AutoencoderKL, VAEConfig.from_pretrained(os.path.join(path, "vae")),
                           os.path.join(path, "vae"), device, dtype)
        te = _load_module(CLIPTextModel, CLIPTextConfig.from_pretrained(os.path.join(path, "text_encoder")),
                          os.path.join(path, "text_encoder"), device, dtype, names=("model", "pytorch_model"))
        tok = AutoTokenizer.from_pretrained(os.path.join(path, "tokenizer"))
        sch = load_scheduler(os.path.join(path, "scheduler"), scheduler)
        return cls(unet, vae, te, tok, sch, vae.config.scaling_factor)

    @classmethod
    def from_tensorized(cls, path: str, device="cpu", dtype=torch.float32, scheduler: str | None = None):
        """``{encoder,vae,unet}.tensors`` + ``{encoder,vae,unet}-config.json`` layout."""
        from transformers import AutoTokenizer
        from ..io.tensors import load_into_module
        stats = {}
        mods = {}
        for prefix, mcls, ccls in (("encoder", CLIPTextModel, CLIPTextConfig), ("vae", AutoencoderKL, VAEConfig),
                                   ("unet", UNet2DConditionModel, UNetConfig)):
            cfg = ccls.from_dict(_read_cfg(os.path.join(path, f"{prefix}-config.json")))
            with torch.device("meta"):
                m = mcls(cfg)
            m = m.to_empty(device=device).to(dtype)
            stats[prefix] = load_into_module(m, os.path.join(path, f"{prefix}.tensors"), device=device)
            mods[prefix] = m
        tdir = os.path.join(path, "tokenizer") if os.path.isdir(os.path.join(path, "tokenizer")) else path
        tok = AutoTokenizer.from_pretrained(tdir)
        sdir = os.path.join(path, "scheduler")
        sch = load_scheduler(sdir if os.path.isdir(sdir) else sd_scheduler_config(), scheduler or "LMSDiscreteScheduler")
        pipe = cls(mods["unet"], mods["vae"], mods["encoder"], tok, sch, mods["vae"].config.scaling_factor)
        pipe.load_stats = stats
        return pipe

    def save_pretrained(self, path: str):
        """diffusers layout (safety_checker / feature_extractor recorded as null:
        the CompVis checker weights are not available offline)."""
        from safetensors.torch import save_file
        os.makedirs(path, exist_ok=True)
        for name, m, cfg, fn in (("unet", self.unet, self.unet.config.to_dict(), "diffusion_pytorch_model"),
                                 ("vae", self.vae, self.vae.config.to_dict(), "diffusion_pytorch_model")):
            d = os.path.join(path, name)
            os.makedirs(d, exist_ok=True)
            with open(os.path.join(d, "config.json"), "w") as f:
                json.dump(cfg, f, indent=2)
            save_file({k: v.detach().contiguous().cpu() for k, v in m.state_dict().items()},
                      os.path.join(d, fn + ".safetensors"), metadata={"format": "pt"})
        self.text_encoder.save_pretrained(os.path.join(path, "text_encoder"))
        self.tokenizer.save_pretrained(os.path.join(path, "tokenizer"))
        self.scheduler.save_pretrained(os.path.join(path, "scheduler"))
        idx = {"_class_name": "StableDiffusionPipeline", "_diffusers_version": "0.14.0",
               "unet": ["diffusers", "UNet2DConditionModel"], "vae": ["diffusers", "AutoencoderKL"],
               "text_encoder": ["transformers", "CLIPTextModel"], "tokenizer": ["transformers", "CLIPTokenizer"],
               "scheduler": ["diffusers", type(self.scheduler).__name__],
               "safety_checker": [None, None], "feature_extractor": [None, None],
               "requires_safety_checker": False}
        with open(os.path.join(path, "model_index.json"), "w") as f:
            json.dump(idx, f, indent=2)

    # -------------------------------------------------------------- encode
    @torch.no_grad()
    def encode_prompt(self, prompts: list[str]) -> torch.Tensor:
        ml = getattr(self.tokenizer, "model_max_length", 77)
        if ml > 1024:
            ml = 77
        tok = self.tokenizer(prompts, padding="max_length", max_length=ml, truncation=True, return_tensors="pt")
        ids = tok.input_ids.to(self.device)
        return self.text_encoder(ids)

    # --------------------------------------------------------------- sample
    @torch.no_grad()
    def __call__(self, prompt, height: int = 512, width: int = 512, num_inference_steps: int = 50,
                 guidance_scale: float = 7.0, negative_prompt=None, generator: torch.Generator | None = None,
                 latents: torch.Tensor | None = None, output_type: str = "pil"):
        prompts = [prompt] if isinstance(prompt, str) else list(prompt)
        B = len(prompts)
        dev, dt = self.device, self.dtype
        cond = self.encode_prompt(prompts)
        cfg = guidance_scale > 1.0
        if cfg:
            neg = negative_prompt or [""] * B
            neg = [neg] * B if isinstance(neg, str) else neg
            ctx = torch.cat([self.encode_prompt(neg), cond])
        else:
            ctx = cond
        sch = self.scheduler
        sch.set_timesteps(num_inference_steps, device=dev)
        f = 2 ** (len(self.vae.config.block_out_channels) - 1)  # 8 for the SD VAE
        shape = (B, self.unet.config.in_channels, height // f, width // f)
        if latents is None:
            latents = torch.randn(shape, generator=generator, device=generator.device if generator else dev,
                                  dtype=torch.float32).to(dev)
        x = latents.to(dev).float() * sch.init_noise_sigma
        run = self._runner()
        if self._fused_sampler_ok(sch, dev, dt):
            x = self._sample_fused(run, sch, x, ctx, guidance_scale if cfg else None)
        else:
            x = self._sample_torch(run, sch, x, ctx, guidance_scale if cfg else None)
        if output_type == "latent":
            return x
        img = self.vae.decode((x / self.scaling_factor).to(dt)).float()
        if output_type == "tensor":
            return img
        from ..data.images import to_pil
        return to_pil(img)

    @staticmethod
    def _fused_sampler_ok(sch, dev, dtype) -> bool:
        import os

        from ..ops import _lib
        from .schedulers import LMSDiscreteScheduler
        return (dev.type == "cuda" and dtype == torch.bfloat16 and isinstance(sch, LMSDiscreteScheduler)
                and _lib.has("kca_sd_lms_step") and os.environ.get("KCA_SD_FUSED_STEP", "1") not in ("0", "false"))

    def _sample_fused(self, run, sch, x, ctx, guidance):
        """LMS / Euler sampling with one fused kernel per step between UNet replays
        (ops/sd_step.py): CFG combine + multistep update + the next scaled bf16
        UNet input, instead of ~15 elementwise launches."""
        from ..ops.sd_step import lms_step
        from .schedulers import EulerDiscreteScheduler
        dev, dt = x.device, self.dtype
        euler = isinstance(sch, EulerDiscreteScheduler)
        order = 1 if euler else 4
        x = x.contiguous(memory_format=torch.channels_last) if x.dim() == 4 else x.contiguous()
        ring = torch.zeros((order, x.numel()), device=dev, dtype=torch.float32)
        sig = sch.sigmas.tolist()
        xin = sch.scale_model_input(torch.cat([x, x]) if guidance is not None else x, sch.timesteps[0]).to(dt)
        xin = xin.contiguous(memory_format=torch.channels_last) if xin.dim() == 4 else xin
        n = len(sch.timesteps)
        for i, t in enumerate(sch.timesteps):
            tt = torch.full((xin.shape[0],), float(t), device=dev)
            eps = run(xin, tt, ctx)
            if eps.dtype != torch.bfloat16:
                eps = eps.to(torch.bfloat16)
            if eps.stride()[1:] != x.stride()[1:]:
                eps = eps.contiguous(memory_format=torch.channels_last) if eps.dim() == 4 else eps.contiguous()
            o = 1 if euler else min(i + 1, order)
            coefs = [sig[i + 1] - sig[i]] if euler else [sch._coef(o, i, j) for j in range(o)]
            last = i + 1 == n
            nxt = None if last else torch.empty_like(xin)
            lms_step(eps, x, ring, coefs, i % order, sig[i], guidance, sch.prediction_type,
                     None if last else 1.0 / (sig[i + 1] ** 2 + 1) ** 0.5, nxt)
            xin = nxt
        return x.contiguous()

    def _sample_torch(self, run, sch, x, ctx, guidance):
        dev, dt = x.device, self.dtype
        cfg = guidance is not None
        guidance_scale = guidance
        for t in sch.timesteps:
            xin = torch.cat([x, x]) if cfg else x
            xin = sch.scale_model_input(xin, t).to(dt)
            tt = torch.full((xin.shape[0],), float(t), device=dev)
            eps = run(xin, tt, ctx).float()
            if cfg:
                eu, ec = eps.chunk(2)
                eps = eu + guidance_scale * (ec - eu)
            x = sch.step(eps, t, x).float()
        return x


def serialize_pipeline(pipe: StableDiffusionPipeline, out_dir: str, dtype: torch.dtype | None = None):
    """Write the tensorized layout (serializer/serialize.py:13-50): encoder/vae/unet
    ``.tensors`` + ``*-config.json`` + tokenizer + scheduler (self-contained:
    the reference relied on writing into an existing diffusers dir)."""
    from ..io.tensors import serialize
    os.makedirs(out_dir, exist_ok=True)
    stats = {}
    for prefix, m, cfg in (("encoder", pipe.text_encoder, pipe.text_encoder.config.to_dict()),
                           ("vae", pipe.vae, pipe.vae.config.to_dict()),
                           ("unet", pipe.unet, pipe.unet.config.to_dict())):
        stats[prefix] = serialize(m, os.path.join(out_dir, f"{prefix}.tensors"), dtype=dtype)
        with open(os.path.join(out_dir, f"{prefix}-config.json"), "w") as f:
            json.dump(cfg, f, indent=2)
    pipe.tokenizer.save_pretrained(out_dir)
    pipe.tokenizer.save_pretrained(os.path.join(out_dir, "tokenizer"))
    pipe.scheduler.save_pretrained(os.path.join(out_dir, "scheduler"))
    return stats
