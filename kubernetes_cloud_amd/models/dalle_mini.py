"""DALL·E mini / mega text-to-image (S12), PyTorch-native on the framework's ops.

The reference serves ``dalle-mini/dalle-mini`` / ``dalle-mega`` through JAX
(online-inference/dalle-mini/model/service.py:75-109: ``DalleBart.generate``
with top-k / top-p / temperature and "super conditioning" ``condition_scale``,
then ``VQModel.decode_code`` of the 256 image tokens into a 256x256 image,
``jax.pmap`` over local devices). There is no JAX on MI355X here, and the
north star excludes a second framework, so the same model family is rebuilt
on this stack:

* ``DalleBart``: BART-style encoder-decoder in the dalle-mini layout --
  learned positions + embedding LayerNorm, NormFormer sub-layer norms (an
  extra LN after attention and inside the FFN), GLU feed-forward
  (``gelu(x W0) * (x W1)`` -> LN -> W2), bias-free linears, final LNs; the
  encoder reads <= 64 text tokens, the decoder emits 256 image tokens of a
  16384-entry VQGAN codebook after a BOS token (id 16384). Attention runs on
  the flash-attention kernels (bidirectional encoder, causal decoder prompt)
  and a KV cache for the token-by-token decode;
* super conditioning: conditional and empty-prompt sequences decode as one
  batch, ``logits = uncond + condition_scale * (cond - uncond)``;
* ``VQGANDecoder``: the taming-transformers f16 decoder (codebook 16384 x 256,
  ch 128, ch_mult (1, 1, 2, 2, 4), 2 res blocks, attention at 16x16) on the
  SD building blocks (fused GroupNorm+SiLU, channels-last convolutions).

Weights: ``load_dalle(dir)`` reads ``config.json`` (dalle-mini field names) and
either the Flax checkpoint the reference's downloader fetches
(``flax_model.msgpack``, decoded without JAX by ``io/flax_msgpack.py`` and
mapped onto these modules by ``dalle_from_flax`` / ``vqgan_from_flax``: Dense
kernels [in, out] -> Linear weights, Conv kernels [kh, kw, in, out] -> OIHW,
LayerNorm/GroupNorm ``scale`` -> weight, scanned (stacked) or per-layer
DalleBart layouts) or a PyTorch ``*.safetensors`` / ``*.bin`` state dict;
otherwise the model is random-init for the given config (benchmarks, tests).
The Flax names follow dalle-mini's modeling code (auto-named ``LayerNorm_k`` /
``FlaxBartAttention_k`` / ``GLU_0`` sub-modules) and vqgan-jax's; no released
checkpoint is in the tree, so parity with the published files is unpinned --
unmatched names are reported, not guessed.
"""
from __future__ import annotations

import dataclasses
import json
import os

import torch
import torch.nn as nn
import torch.nn.functional as F

from .. import ops
from .unet import ResnetBlock2D, Upsample2D, to_channels_last


@dataclasses.dataclass
class DalleBartConfig:
    encoder_vocab_size: int = 50264
    image_vocab_size: int = 16384
    d_model: int = 1024
    encoder_layers: int = 12
    decoder_layers: int = 12
    encoder_attention_heads: int = 16
    decoder_attention_heads: int = 16
    encoder_ffn_dim: int = 2730
    decoder_ffn_dim: int = 2730
    max_text_length: int = 64
    image_length: int = 256
    ln_eps: float = 1e-5

    @property
    def bos_token_id(self) -> int:
        return self.image_vocab_size

    @classmethod
    def from_dict(cls, d: dict) -> "DalleBartConfig":
        names = {f.name for f in dataclasses.fields(cls)}
        return cls(**{k: v for k, v in d.items() if k in names})

    @classmethod
    def mega(cls) -> "DalleBartConfig":
        return cls(d_model=2048, encoder_layers=24, decoder_layers=24, encoder_attention_heads=32,
                   decoder_attention_heads=32, encoder_ffn_dim=4096, decoder_ffn_dim=4096)


class _Attn(nn.Module):
    def __init__(self, d: int, heads: int):
        super().__init__()
        self.h = heads
        self.q_proj = nn.Linear(d, d, bias=False)
        self.k_proj = nn.Linear(d, d, bias=False)
        self.v_proj = nn.Linear(d, d, bias=False)
        self.out_proj = nn.Linear(d, d, bias=False)

    def forward(self, x, ctx=None, causal=False, cache=None):
        """cache: dict with 'k','v' [B, T, H, Dh] appended in place (decode)."""
        B, S, d = x.shape
        c = x if ctx is None else ctx
        q = self.q_proj(x).view(B, S, self.h, -1)
        if cache is not None and ctx is not None and "k" in cache:  # cross-attention: encoder K/V cached once
            k, v = cache["k"], cache["v"]
        else:
            k = self.k_proj(c).view(B, c.shape[1], self.h, -1)
            v = self.v_proj(c).view(B, c.shape[1], self.h, -1)
            if cache is not None:
                if ctx is None and "k" in cache:
                    k = torch.cat([cache["k"], k], 1)
                    v = torch.cat([cache["v"], v], 1)
                cache["k"], cache["v"] = k, v
        if S == 1 and cache is not None:  # one decode token against the cache
            s = torch.einsum("bqhd,bkhd->bhqk", q.float(), k.float()) / (q.shape[-1] ** 0.5)
            o = torch.einsum("bhqk,bkhd->bqhd", s.softmax(-1), v.float()).to(x.dtype)
        else:
            o = ops.flash_attention(q, k, v, causal=causal)
        return self.out_proj(o.reshape(B, S, d))


class _GLU(nn.Module):
    def __init__(self, d: int, ffn: int, eps: float):
        super().__init__()
        self.ln0 = nn.LayerNorm(d, eps=eps)
        self.fc0 = nn.Linear(d, ffn, bias=False)
        self.fc1 = nn.Linear(d, ffn, bias=False)
        self.ln1 = nn.LayerNorm(ffn, eps=eps)
        self.fc2 = nn.Linear(ffn, d, bias=False)

    def forward(self, x):
        h = ops.layer_norm(x, self.ln0.weight, self.ln0.bias, self.ln0.eps)
        h = F.gelu(self.fc0(h).float()).to(x.dtype) * self.fc1(h)
        return self.fc2(_ln(self.ln1, h))


def _ln(m: nn.LayerNorm, x):
    if x.shape[-1] % 8:  # dalle-mini's GLU width 2730: outside the 16-B vector LN kernel
        return F.layer_norm(x.float(), x.shape[-1:], m.weight.float(), m.bias.float(), m.eps).to(x.dtype)
    return ops.layer_norm(x, m.weight, m.bias, m.eps)


class _EncLayer(nn.Module):
    def __init__(self, c: DalleBartConfig):
        super().__init__()
        d = c.d_model
        self.pre_self_attn_layer_norm = nn.LayerNorm(d, eps=c.ln_eps)
        self.self_attn = _Attn(d, c.encoder_attention_heads)
        self.self_attn_layer_norm = nn.LayerNorm(d, eps=c.ln_eps)  # NormFormer post-attention LN
        self.glu = _GLU(d, c.encoder_ffn_dim, c.ln_eps)

    def forward(self, x):
        x = x + _ln(self.self_attn_layer_norm, self.self_attn(_ln(self.pre_self_attn_layer_norm, x)))
        return x + self.glu(x)


class _DecLayer(nn.Module):
    def __init__(self, c: DalleBartConfig):
        super().__init__()
        d = c.d_model
        self.pre_self_attn_layer_norm = nn.LayerNorm(d, eps=c.ln_eps)
        self.self_attn = _Attn(d, c.decoder_attention_heads)
        self.self_attn_layer_norm = nn.LayerNorm(d, eps=c.ln_eps)
        self.pre_encoder_attn_layer_norm = nn.LayerNorm(d, eps=c.ln_eps)
        self.encoder_attn = _Attn(d, c.decoder_attention_heads)
        self.encoder_attn_layer_norm = nn.LayerNorm(d, eps=c.ln_eps)
        self.glu = _GLU(d, c.decoder_ffn_dim, c.ln_eps)

    def forward(self, x, enc, cache=None):
        sc = cache["self"] if cache is not None else None
        cc = cache["cross"] if cache is not None else None
        x = x + _ln(self.self_attn_layer_norm,
                    self.self_attn(_ln(self.pre_self_attn_layer_norm, x), causal=True, cache=sc))
        x = x + _ln(self.encoder_attn_layer_norm,
                    self.encoder_attn(_ln(self.pre_encoder_attn_layer_norm, x), ctx=enc, cache=cc))
        return x + self.glu(x)


class DalleBart(nn.Module):
    def __init__(self, config: DalleBartConfig):
        super().__init__()
        c = self.config = config
        d = c.d_model
        self.embed_tokens = nn.Embedding(c.encoder_vocab_size, d)
        self.embed_positions = nn.Embedding(c.max_text_length, d)
        self.layernorm_embedding = nn.LayerNorm(d, eps=c.ln_eps)
        self.encoder_layers = nn.ModuleList([_EncLayer(c) for _ in range(c.encoder_layers)])
        self.encoder_final_ln = nn.LayerNorm(d, eps=c.ln_eps)
        self.dec_embed_tokens = nn.Embedding(c.image_vocab_size + 1, d)
        self.dec_embed_positions = nn.Embedding(c.image_length + 1, d)
        self.dec_layernorm_embedding = nn.LayerNorm(d, eps=c.ln_eps)
        self.decoder_layers = nn.ModuleList([_DecLayer(c) for _ in range(c.decoder_layers)])
        self.decoder_final_ln = nn.LayerNorm(d, eps=c.ln_eps)
        self.lm_head = nn.Linear(d, c.image_vocab_size + 1, bias=False)

    def encode(self, input_ids: torch.Tensor) -> torch.Tensor:
        pos = torch.arange(input_ids.shape[1], device=input_ids.device)
        x = _ln(self.layernorm_embedding, self.embed_tokens(input_ids) + self.embed_positions(pos))
        for layer in self.encoder_layers:
            x = layer(x)
        return _ln(self.encoder_final_ln, x)

    def decode(self, tokens, enc, start: int = 0, caches=None):
        pos = torch.arange(start, start + tokens.shape[1], device=tokens.device)
        x = _ln(self.dec_layernorm_embedding, self.dec_embed_tokens(tokens) + self.dec_embed_positions(pos))
        for i, layer in enumerate(self.decoder_layers):
            x = layer(x, enc, None if caches is None else caches[i])
        return self.lm_head(_ln(self.decoder_final_ln, x))

    def forward(self, input_ids, decoder_input_ids):
        return self.decode(decoder_input_ids, self.encode(input_ids))

    @torch.no_grad()
    def generate(self, input_ids: torch.Tensor, uncond_ids: torch.Tensor | None = None, top_k: int = 50,
                 top_p: float = 1.0, temperature: float = 1.0, condition_scale: float = 10.0,
                 generator: torch.Generator | None = None) -> torch.Tensor:
        """Sample ``image_length`` codebook indices per prompt (BOS excluded)."""
        c = self.config
        B = input_ids.shape[0]
        sup = uncond_ids is not None and condition_scale != 1.0
        ids = torch.cat([input_ids, uncond_ids]) if sup else input_ids
        enc = self.encode(ids)
        caches = [{"self": {}, "cross": {}} for _ in self.decoder_layers]
        tok = torch.full((ids.shape[0], 1), c.bos_token_id, dtype=torch.long, device=ids.device)
        out = []
        for t in range(c.image_length):
            logits = self.decode(tok, enc, start=t, caches=caches)[:, -1].float()
            if sup:
                lc, lu = logits[:B], logits[B:]
                logits = lu + condition_scale * (lc - lu)
            nxt = sample_next(logits, top_k, top_p, temperature, generator, ban=c.bos_token_id)
            out.append(nxt)
            tok = torch.cat([nxt, nxt]) if sup else nxt
            tok = tok[:, None]
        return torch.stack(out, 1)


def sample_next(logits: torch.Tensor, top_k: int, top_p: float, temperature: float, generator=None,
                ban: int | None = None) -> torch.Tensor:
    """HF-style warpers (temperature -> top-k -> top-p) + multinomial; greedy at temperature 0."""
    if ban is not None:
        logits[:, ban] = float("-inf")
    if temperature <= 0:
        return logits.argmax(-1)
    logits = logits / temperature
    if top_k and top_k > 0:
        kth = torch.topk(logits, min(top_k, logits.shape[-1]), dim=-1).values[:, -1:]
        logits = logits.masked_fill(logits < kth, float("-inf"))
    if top_p < 1.0:
        srt, idx = torch.sort(logits, descending=True, dim=-1)
        cum = srt.softmax(-1).cumsum(-1)
        drop = cum - srt.softmax(-1) > top_p
        srt = srt.masked_fill(drop, float("-inf"))
        logits = torch.full_like(logits, float("-inf")).scatter(-1, idx, srt)
    probs = logits.softmax(-1)
    return torch.multinomial(probs, 1, generator=generator)[:, 0]


# ---------------------------------------------------------------- VQGAN f16
@dataclasses.dataclass
class VQGANConfig:
    n_embed: int = 16384
    embed_dim: int = 256
    z_channels: int = 256
    ch: int = 128
    ch_mult: tuple = (1, 1, 2, 2, 4)
    num_res_blocks: int = 2
    attn_resolutions: tuple = (16,)
    resolution: int = 256
    out_ch: int = 3

    @classmethod
    def from_dict(cls, d: dict) -> "VQGANConfig":
        names = {f.name for f in dataclasses.fields(cls)}
        kw = {k: tuple(v) if isinstance(v, list) else v for k, v in d.items() if k in names}
        return cls(**kw)


class _VQAttn(nn.Module):
    def __init__(self, ch):
        super().__init__()
        self.norm = nn.GroupNorm(32, ch, eps=1e-6)
        self.q = nn.Conv2d(ch, ch, 1)
        self.k = nn.Conv2d(ch, ch, 1)
        self.v = nn.Conv2d(ch, ch, 1)
        self.proj_out = nn.Conv2d(ch, ch, 1)

    def forward(self, x):
        B, C, H, W = x.shape
        h = ops.group_norm(x, 32, self.norm.weight, self.norm.bias, self.norm.eps)
        t = h.permute(0, 2, 3, 1).reshape(B, H * W, C)
        lin = (lambda m, z: F.linear(z, m.weight.reshape(C, C), m.bias))
        q, k, v = lin(self.q, t), lin(self.k, t), lin(self.v, t)
        if C <= 256:
            o = ops.flash_attention(q[:, :, None], k[:, :, None], v[:, :, None])[:, :, 0]
        else:
            s = torch.einsum("bqc,bkc->bqk", q.float(), k.float()) / (C ** 0.5)
            o = torch.einsum("bqk,bkc->bqc", s.softmax(-1), v.float()).to(q.dtype)
        o = lin(self.proj_out, o)
        return x + o.view(B, H, W, C).permute(0, 3, 1, 2)


class VQGANDecoder(nn.Module):
    """``decode_code(indices [B, h*w]) -> images [B, 3, 16h, 16w]`` in [0, 1]."""

    def __init__(self, config: VQGANConfig):
        super().__init__()
        c = self.config = config
        self.embedding = nn.Embedding(c.n_embed, c.embed_dim)
        self.post_quant_conv = nn.Conv2d(c.embed_dim, c.z_channels, 1)
        chs = [c.ch * m for m in c.ch_mult]
        block_in = chs[-1]
        curr = c.resolution // 2 ** (len(c.ch_mult) - 1)
        self.conv_in = nn.Conv2d(c.z_channels, block_in, 3, padding=1)
        self.mid = nn.ModuleList([ResnetBlock2D(block_in, block_in, 0, 32, 1e-6), _VQAttn(block_in),
                                  ResnetBlock2D(block_in, block_in, 0, 32, 1e-6)])
        ups = []
        for lvl in reversed(range(len(c.ch_mult))):
            blocks = []
            out = chs[lvl]
            for _ in range(c.num_res_blocks + 1):
                blocks.append(ResnetBlock2D(block_in, out, 0, 32, 1e-6))
                block_in = out
                if curr in c.attn_resolutions:
                    blocks.append(_VQAttn(block_in))
            if lvl != 0:
                blocks.append(Upsample2D(block_in))
                curr *= 2
            ups.append(nn.ModuleList(blocks))
        self.up = nn.ModuleList(ups)
        from .unet import GroupNorm
        self.norm_out = GroupNorm(32, block_in, 1e-6, silu=True)
        self.conv_out = nn.Conv2d(block_in, c.out_ch, 3, padding=1)
        self.channels_last = False

    def decode_code(self, indices: torch.Tensor) -> torch.Tensor:
        B, n = indices.shape
        side = int(round(n ** 0.5))
        z = self.embedding(indices).view(B, side, side, -1).permute(0, 3, 1, 2)
        z = z.contiguous(memory_format=torch.channels_last) if self.channels_last else z.contiguous()
        x = self.conv_in(self.post_quant_conv(z))
        for m in self.mid:
            x = m(x)
        for blocks in self.up:
            for m in blocks:
                x = m(x)
        x = self.conv_out(self.norm_out(x)).contiguous()
        return ((x.float() + 1.0) / 2.0).clamp(0.0, 1.0)


# ------------------------------------------------------------- Flax checkpoints
def _dalle_flax_names(c: DalleBartConfig):
    """(our key prefix, Flax path, kind) for every DalleBart tensor; kind: dense (kernel, transposed),
    embed, ln (scale/bias). Layer paths use '{L}' for the per-layer part (layers/{i} or scanned)."""
    out = [("embed_tokens", "model/encoder/embed_tokens", "embed"),
           ("embed_positions", "model/encoder/embed_positions", "embed"),
           ("layernorm_embedding", "model/encoder/layernorm_embedding", "ln"),
           ("encoder_final_ln", "model/encoder/final_ln", "ln"),
           ("dec_embed_tokens", "model/decoder/embed_tokens", "embed"),
           ("dec_embed_positions", "model/decoder/embed_positions", "embed"),
           ("dec_layernorm_embedding", "model/decoder/layernorm_embedding", "ln"),
           ("decoder_final_ln", "model/decoder/final_ln", "ln"),
           ("lm_head", "lm_head", "dense")]
    glu = [("glu.ln0", "GLU_0/LayerNorm_0", "ln"), ("glu.fc0", "GLU_0/Dense_0", "dense"),
           ("glu.fc1", "GLU_0/Dense_1", "dense"), ("glu.ln1", "GLU_0/LayerNorm_1", "ln"),
           ("glu.fc2", "GLU_0/Dense_2", "dense")]

    def attn(ours, flax):
        return [(f"{ours}.{n}", f"{flax}/{n}", "dense") for n in ("q_proj", "k_proj", "v_proj", "out_proj")]
    enc = [("pre_self_attn_layer_norm", "LayerNorm_0", "ln"), *attn("self_attn", "FlaxBartAttention_0"),
           ("self_attn_layer_norm", "LayerNorm_1", "ln"), *glu]
    dec = [("pre_self_attn_layer_norm", "LayerNorm_0", "ln"), *attn("self_attn", "FlaxBartAttention_0"),
           ("self_attn_layer_norm", "LayerNorm_1", "ln"), ("pre_encoder_attn_layer_norm", "LayerNorm_2", "ln"),
           *attn("encoder_attn", "FlaxBartAttention_1"), ("encoder_attn_layer_norm", "LayerNorm_3", "ln"), *glu]
    layers = [("encoder_layers", "model/encoder/layers", "FlaxBartEncoderLayers", c.encoder_layers, enc),
              ("decoder_layers", "model/decoder/layers", "FlaxBartDecoderLayers", c.decoder_layers, dec)]
    return out, layers


def _flax_get(flat: dict, path: str, kind: str, layer: int | None = None, stacked: bool = False):
    """{'weight': t, 'bias': t?} of one module from a flat Flax dict (None when absent)."""
    def g(name):
        t = flat.get(f"{path}/{name}")
        if t is not None and stacked:
            t = t[layer]
        return t
    if kind == "embed":
        t = g("embedding")
        return None if t is None else {"weight": t}
    if kind == "dense":
        t = g("kernel")
        if t is None:
            return None
        d = {"weight": t.t().contiguous()}
        b = g("bias")
        if b is not None:
            d["bias"] = b
        return d
    if kind == "conv":
        t = g("kernel")
        if t is None:
            return None
        d = {"weight": t.permute(3, 2, 0, 1).contiguous()}
        b = g("bias")
        if b is not None:
            d["bias"] = b
        return d
    sc, b = g("scale"), g("bias")  # ln / gn: a norm built with use_scale=False has no scale
    if sc is None and b is None:
        return None
    d = {}
    if sc is not None:
        d["weight"] = sc
    if b is not None:
        d["bias"] = b
    return d


def _strip_root(flat: dict) -> dict:
    if flat and all(k.startswith("params/") for k in flat):
        return {k[len("params/"):]: v for k, v in flat.items()}
    return flat


def dalle_from_flax(flat: dict, c: DalleBartConfig) -> tuple[dict, list]:
    """Flax DalleBart params (flattened 'a/b/c' keys) -> (our state dict, unmatched Flax keys).
    Per-layer ('layers/{i}/...') and scanned ('layers/FlaxBart{Encoder,Decoder}Layers/...', leading
    layer axis) layouts; a final LayerNorm stored as the last layer's extra norm (LayerNorm_2 in an
    encoder layer, LayerNorm_4 in a decoder layer) is accepted for ``final_ln``."""
    flat = _strip_root(flat)
    used: set = set()
    sd: dict = {}

    def put(ours, mod):
        for k, v in mod.items():
            sd[f"{ours}.{k}"] = v

    def take(path, kind, ours, layer=None, stacked=False):
        mod = _flax_get(flat, path, kind, layer, stacked)
        if mod is not None:
            put(ours, mod)
            used.update(k for k in flat if k.startswith(path + "/"))
        return mod is not None

    top, layers = _dalle_flax_names(c)
    for ours, path, kind in top:
        if not take(path, kind, ours) and ours.endswith("final_ln"):
            side = "encoder" if ours.startswith("encoder") else "decoder"
            n = c.encoder_layers if side == "encoder" else c.decoder_layers
            extra = "LayerNorm_2" if side == "encoder" else "LayerNorm_4"
            if not take(f"model/{side}/layers/{n - 1}/{extra}", "ln", ours):
                scan = f"model/{side}/layers/FlaxBart{side.capitalize()}Layers/{extra}"
                take(scan, "ln", ours, n - 1, True)
    for ours_root, root, scan_name, n, subs in layers:
        stacked = any(k.startswith(f"{root}/{scan_name}/") for k in flat)
        for i in range(n):
            for ours, sub, kind in subs:
                path = f"{root}/{scan_name}/{sub}" if stacked else f"{root}/{i}/{sub}"
                take(path, kind, f"{ours_root}.{i}.{ours}", i, stacked)
    return sd, sorted(k for k in flat if k not in used)


def dalle_to_flax(model: "DalleBart", stacked: bool = False) -> dict:
    """Our DalleBart -> flat Flax params in the layout ``dalle_from_flax`` reads (tests, exports)."""
    c = model.config
    sd = {k: v.detach().cpu() for k, v in model.state_dict().items()}

    def vals(ours, kind):
        w, b = sd.get(f"{ours}.weight"), sd.get(f"{ours}.bias")
        if kind == "embed":
            return {"embedding": w}
        if kind == "dense":
            return {"kernel": w.t().contiguous(), **({"bias": b} if b is not None else {})}
        return {"scale": w, "bias": b}
    flat = {}
    top, layers = _dalle_flax_names(c)
    for ours, path, kind in top:
        for k, v in vals(ours, kind).items():
            flat[f"{path}/{k}"] = v
    for ours_root, root, scan_name, n, subs in layers:
        for ours, sub, kind in subs:
            per = [vals(f"{ours_root}.{i}.{ours}", kind) for i in range(n)]
            for k in per[0]:
                if stacked:
                    flat[f"{root}/{scan_name}/{sub}/{k}"] = torch.stack([d[k] for d in per])
                else:
                    for i in range(n):
                        flat[f"{root}/{i}/{sub}/{k}"] = per[i][k]
    return flat


def _vqgan_flax_names(m: "VQGANDecoder"):
    """(our module prefix, Flax path, kind) for the vqgan-jax VQModel decoder side."""
    c = m.config
    out = [("embedding", "quantize/embedding", "embed"), ("post_quant_conv", "post_quant_conv", "conv"),
           ("conv_in", "decoder/conv_in", "conv"), ("norm_out", "decoder/norm_out", "ln"),
           ("conv_out", "decoder/conv_out", "conv")]

    def res(ours, flax, has_sc):
        r = [(f"{ours}.norm1", f"{flax}/norm1", "ln"), (f"{ours}.conv1", f"{flax}/conv1", "conv"),
             (f"{ours}.norm2", f"{flax}/norm2", "ln"), (f"{ours}.conv2", f"{flax}/conv2", "conv")]
        if has_sc:
            r.append((f"{ours}.conv_shortcut", f"{flax}/nin_shortcut", "conv"))
        return r

    def att(ours, flax):
        return [(f"{ours}.{n}", f"{flax}/{n}", "ln" if n == "norm" else "conv")
                for n in ("norm", "q", "k", "v", "proj_out")]
    out += res("mid.0", "decoder/mid/block_1", m.mid[0].conv_shortcut is not None)
    out += att("mid.1", "decoder/mid/attn_1")
    out += res("mid.2", "decoder/mid/block_2", m.mid[2].conv_shortcut is not None)
    L = len(c.ch_mult)
    for ui, blocks in enumerate(m.up):
        lvl = L - 1 - ui  # our up[0] is the lowest resolution; vqgan-jax's up_{lvl} is indexed by level
        j_res = j_att = 0
        for bi, blk in enumerate(blocks):
            ours = f"up.{ui}.{bi}"
            if isinstance(blk, ResnetBlock2D):
                out += res(ours, f"decoder/up_{lvl}/block_{j_res}", blk.conv_shortcut is not None)
                j_res += 1
            elif isinstance(blk, _VQAttn):
                out += att(ours, f"decoder/up_{lvl}/attn_{j_att}")
                j_att += 1
            else:  # Upsample2D
                out.append((f"{ours}.conv", f"decoder/up_{lvl}/upsample/conv", "conv"))
    return out


def vqgan_from_flax(flat: dict, m: "VQGANDecoder") -> tuple[dict, list]:
    """Flax VQModel params -> (our VQGANDecoder state dict, unmatched Flax keys; the VQGAN
    encoder / quant_conv halves are not used by decode_code and are reported there)."""
    flat = _strip_root(flat)
    sd, used = {}, set()
    for ours, path, kind in _vqgan_flax_names(m):
        mod = _flax_get(flat, path, kind)
        if mod is not None:
            for k, v in mod.items():
                sd[f"{ours}.{k}"] = v
            used.update(k for k in flat if k.startswith(path + "/"))
    return sd, sorted(k for k in flat if k not in used)


def vqgan_to_flax(m: "VQGANDecoder") -> dict:
    sd = {k: v.detach().cpu() for k, v in m.state_dict().items()}
    flat = {}
    for ours, path, kind in _vqgan_flax_names(m):
        w, b = sd[f"{ours}.weight"], sd.get(f"{ours}.bias")
        if kind == "embed":
            flat[f"{path}/embedding"] = w
        elif kind == "conv":
            flat[f"{path}/kernel"] = w.permute(2, 3, 1, 0).contiguous()
            flat[f"{path}/bias"] = b
        else:
            flat[f"{path}/scale"], flat[f"{path}/bias"] = w, b
    return flat


def _load_flax(module: nn.Module, path: str) -> bool:
    f = os.path.join(path, "flax_model.msgpack")
    if not os.path.exists(f):
        return False
    from ..io import flax_msgpack
    flat = flax_msgpack.flatten(flax_msgpack.read(f))
    if isinstance(module, DalleBart):
        sd, extra = dalle_from_flax(flat, module.config)
    else:
        sd, extra = vqgan_from_flax(flat, module)
    import logging
    log = logging.getLogger("kca.dalle")
    own = module.state_dict()
    for k, v in sd.items():  # norms saved without a scale keep their ones
        if k in own:
            own[k] = v.to(own[k].dtype).reshape(own[k].shape)
    missing = [k for k in own if k not in sd]
    if missing:
        log.warning("%s: %d parameters not in the Flax checkpoint (kept as initialised), e.g. %s", f,
                    len(missing), missing[:4])
    if extra:
        log.info("%s: %d Flax tensors unused (e.g. %s)", f, len(extra), extra[:4])
    module.load_state_dict(own)
    return True


def _load_state(module: nn.Module, path: str) -> bool:
    if _load_flax(module, path):
        return True
    for name in ("model.safetensors", "pytorch_model.safetensors", "pytorch_model.bin", "model.bin"):
        f = os.path.join(path, name)
        if os.path.exists(f):
            if f.endswith(".safetensors"):
                from safetensors.torch import load_file
                sd = load_file(f)
            else:
                sd = torch.load(f, map_location="cpu", weights_only=True)
            module.load_state_dict(sd, strict=False)
            return True
    return False


def load_dalle(path: str | None, device="cpu", dtype=torch.float32, config: DalleBartConfig | None = None,
               vq_config: VQGANConfig | None = None, seed: int = 0):
    """(DalleBart, VQGANDecoder) from a model directory (``config.json`` +
    PyTorch weights, VQGAN under ``vqgan/``), or random-init for the configs."""
    torch.manual_seed(seed)
    cfg, vcfg = config, vq_config
    if path and os.path.exists(os.path.join(path, "config.json")):
        with open(os.path.join(path, "config.json")) as f:
            cfg = DalleBartConfig.from_dict(json.load(f))
    vq_dir = os.path.join(path, "vqgan") if path else None
    if vq_dir and os.path.exists(os.path.join(vq_dir, "config.json")):
        with open(os.path.join(vq_dir, "config.json")) as f:
            vcfg = VQGANConfig.from_dict(json.load(f))
    model = DalleBart(cfg or DalleBartConfig())
    vq = VQGANDecoder(vcfg or VQGANConfig())
    if path:
        _load_state(model, path)
    if vq_dir:
        _load_state(vq, vq_dir)
    model = model.to(device=device, dtype=dtype).eval()
    vq = vq.to(device=device, dtype=dtype).eval()
    if vq.embedding.weight.is_cuda:
        to_channels_last(vq)
    return model, vq


__all__ = ["DalleBartConfig", "DalleBart", "VQGANConfig", "VQGANDecoder", "load_dalle", "sample_next",
           "dalle_from_flax", "dalle_to_flax", "vqgan_from_flax", "vqgan_to_flax"]
