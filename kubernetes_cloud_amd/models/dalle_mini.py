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

Weights: ``from_pretrained(dir)`` reads ``config.json`` (dalle-mini field names)
and a PyTorch ``*.safetensors`` / ``*.bin`` state dict when present (the Flax
msgpack checkpoints need a one-off conversion outside this image); otherwise
the model is random-init for the given config (benchmarks, tests).
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


def _load_state(module: nn.Module, path: str) -> bool:
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


__all__ = ["DalleBartConfig", "DalleBart", "VQGANConfig", "VQGANDecoder", "load_dalle", "sample_next"]
