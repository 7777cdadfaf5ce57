"""AutoencoderKL (SD VAE) with diffusers-compatible parameter names.

Encoder used by the SD trainer to get latents (sd-finetuner/finetuner.py:
470-473: ``vae.encode(px).latent_dist.sample() * 0.18215``); decoder used by
the txt2img predictor (K20 + the VAE decode of service.py:245-252). GroupNorm
(+SiLU) run on the native kernel; the mid-block single-head attention
(512 channels over 64x64 tokens at 512 px) on the native flash kernel.
"""
from __future__ import annotations

import dataclasses
import json
import os

import torch
import torch.nn as nn
import torch.nn.functional as F

from .. import ops
from .unet import Downsample2D, GroupNorm, ResnetBlock2D, Upsample2D

L_SCALE_FACTOR = 0.18215  # sd-finetuner/finetuner.py:42


@dataclasses.dataclass
class VAEConfig:
    in_channels: int = 3
    out_channels: int = 3
    latent_channels: int = 4
    block_out_channels: tuple = (128, 256, 512, 512)
    layers_per_block: int = 2
    norm_num_groups: int = 32
    scaling_factor: float = L_SCALE_FACTOR
    sample_size: int = 512
    raw: dict = dataclasses.field(default_factory=dict, repr=False)

    @classmethod
    def from_dict(cls, d: dict) -> "VAEConfig":
        kw = {f.name: (tuple(d[f.name]) if isinstance(d[f.name], list) else d[f.name])
              for f in dataclasses.fields(cls) if f.name in d and f.name != "raw"}
        return cls(raw=dict(d), **kw)

    @classmethod
    def from_pretrained(cls, path: str) -> "VAEConfig":
        with open(os.path.join(path, "config.json")) as f:
            return cls.from_dict(json.load(f))

    def to_dict(self):
        d = dict(self.raw) if self.raw else {"_class_name": "AutoencoderKL"}
        for f in dataclasses.fields(self):
            if f.name != "raw":
                v = getattr(self, f.name)
                d[f.name] = list(v) if isinstance(v, tuple) else v
        return d


def _wide_head_attention(q, k, v, scale):
    """Single-head attention over [B, S, C] with C > 256 (the VAE mid-block,
    C = 512, S = 4096 at 512 px). Inference: the 512-wide LDS-DMA flash kernel
    (ops.attention.wide_head_attention; no [B, S, S] scores). Otherwise (autograd,
    odd shapes, a flagged softmax overflow) bf16 operands on the MFMA GEMM path
    with the logits produced in fp32 (``out_dtype``) and an fp32 softmax."""
    global _BMM_OUT_DTYPE
    if _FLASH_WIDE:
        o = ops.attention.wide_head_attention(q, k, v, scale)
        if o is not None:
            return o
    if q.is_cuda and q.dtype == torch.bfloat16 and _BMM_OUT_DTYPE is not False:
        try:  # aten::bmm.dtype (bf16 in, fp32 out) is a GPU-only kernel
            s = torch.bmm(q, k.transpose(1, 2), out_dtype=torch.float32)
            _BMM_OUT_DTYPE = True
        except (TypeError, RuntimeError, NotImplementedError):
            _BMM_OUT_DTYPE = False
        else:
            p = torch.softmax(s.mul_(scale), dim=-1).to(v.dtype)
            return torch.bmm(p, v)
    s = torch.einsum("bqc,bkc->bqk", q.float(), k.float()) * scale
    return torch.einsum("bqk,bkc->bqc", s.softmax(-1), v.float()).to(q.dtype)


_BMM_OUT_DTYPE = None  # probed on the first GPU call
_FLASH_WIDE = os.environ.get("KCA_VAE_FLASH", "1") not in ("0", "false")  # A/B knob


class VAEAttention(nn.Module):
    """diffusers mid-block Attention: group_norm + to_q/k/v + to_out.0, 1 head."""

    def __init__(self, ch, groups):
        super().__init__()
        self.group_norm = nn.GroupNorm(groups, ch, eps=1e-6)
        self.to_q = nn.Linear(ch, ch)
        self.to_k = nn.Linear(ch, ch)
        self.to_v = nn.Linear(ch, ch)
        self.to_out = nn.ModuleList([nn.Linear(ch, ch), nn.Dropout(0.0)])

    def forward(self, x):
        B, C, H, W = x.shape
        h = ops.group_norm(x, self.group_norm.num_groups, self.group_norm.weight, self.group_norm.bias,
                           self.group_norm.eps)
        h = h.reshape(B, C, H * W).transpose(1, 2)
        q, k, v = self.to_q(h), self.to_k(h), self.to_v(h)
        if C <= 256:
            o = ops.flash_attention(q[:, :, None], k[:, :, None], v[:, :, None], causal=False)[:, :, 0]
        else:  # head_dim 512: the wide flash kernel (inference) or two GEMMs around an fp32 softmax
            o = _wide_head_attention(q, k, v, C ** -0.5)
        o = self.to_out[0](o)
        return x + o.transpose(1, 2).reshape(B, C, H, W)


class _Mid(nn.Module):
    def __init__(self, ch, groups):
        super().__init__()
        self.attentions = nn.ModuleList([VAEAttention(ch, groups)])
        self.resnets = nn.ModuleList([ResnetBlock2D(ch, ch, 0, groups, 1e-6), ResnetBlock2D(ch, ch, 0, groups, 1e-6)])

    def forward(self, x):
        x = self.resnets[0](x)
        x = self.attentions[0](x)
        return self.resnets[1](x)


class _DownEnc(nn.Module):
    def __init__(self, cin, cout, n, groups, add_down):
        super().__init__()
        self.resnets = nn.ModuleList([ResnetBlock2D(cin if i == 0 else cout, cout, 0, groups, 1e-6) for i in range(n)])
        self.downsamplers = nn.ModuleList([Downsample2D(cout, pad=0)]) if add_down else None

    def forward(self, x, in_bias=None):
        for i, r in enumerate(self.resnets):
            x = r(x, None, in_bias) if i == 0 and in_bias is not None else r(x)
        if self.downsamplers is not None:
            x = self.downsamplers[0](x)
        return x


class _UpDec(nn.Module):
    def __init__(self, cin, cout, n, groups, add_up):
        super().__init__()
        self.resnets = nn.ModuleList([ResnetBlock2D(cin if i == 0 else cout, cout, 0, groups, 1e-6) for i in range(n)])
        self.upsamplers = nn.ModuleList([Upsample2D(cout)]) if add_up else None

    def forward(self, x):
        for r in self.resnets:
            x = r(x)
        if self.upsamplers is not None:
            x = self.upsamplers[0](x)
        return x


class Encoder(nn.Module):
    def __init__(self, c: VAEConfig):
        super().__init__()
        ch = c.block_out_channels
        g = c.norm_num_groups
        self.conv_in = nn.Conv2d(c.in_channels, ch[0], 3, padding=1)
        blocks, prev = [], ch[0]
        for i, o in enumerate(ch):
            blocks.append(_DownEnc(prev, o, c.layers_per_block, g, i < len(ch) - 1))
            prev = o
        self.down_blocks = nn.ModuleList(blocks)
        self.mid_block = _Mid(ch[-1], g)
        self.conv_norm_out = GroupNorm(g, ch[-1], 1e-6, silu=True)
        self.conv_out = nn.Conv2d(ch[-1], 2 * c.latent_channels, 3, padding=1)

    def forward(self, x):
        if (not torch.is_grad_enabled() and x.is_cuda and x.dtype == torch.bfloat16 and self.conv_in.bias is not None
                and x.is_contiguous(memory_format=torch.channels_last)):
            # conv_in's bias rides in the first ResNet block (its GroupNorm's add and the residual add)
            # instead of a broadcast pass over the full-resolution output (16 x 128 x 512^2 at DreamBooth
            # batch: 0.43 ms)
            x = F.conv2d(x, self.conv_in.weight, None, padding=1)
            x = self.down_blocks[0](x, in_bias=self.conv_in.bias)
            rest = self.down_blocks[1:]
        else:
            x = self.conv_in(x)
            rest = self.down_blocks
        for b in rest:
            x = b(x)
        x = self.mid_block(x)
        return self.conv_out(self.conv_norm_out(x))


class Decoder(nn.Module):
    def __init__(self, c: VAEConfig):
        super().__init__()
        ch = list(reversed(c.block_out_channels))
        g = c.norm_num_groups
        self.conv_in = nn.Conv2d(c.latent_channels, ch[0], 3, padding=1)
        self.mid_block = _Mid(ch[0], g)
        blocks, prev = [], ch[0]
        for i, o in enumerate(ch):
            blocks.append(_UpDec(prev, o, c.layers_per_block + 1, g, i < len(ch) - 1))
            prev = o
        self.up_blocks = nn.ModuleList(blocks)
        self.conv_norm_out = GroupNorm(g, ch[-1], 1e-6, silu=True)
        self.conv_out = nn.Conv2d(ch[-1], c.out_channels, 3, padding=1)

    def forward(self, z):
        x = self.conv_in(z)
        x = self.mid_block(x)
        for b in self.up_blocks:
            x = b(x)
        return self.conv_out(self.conv_norm_out(x))


class DiagonalGaussian:
    def __init__(self, moments: torch.Tensor):
        self.mean, logvar = moments.chunk(2, dim=1)
        self.logvar = logvar.clamp(-30.0, 20.0)
        self.std = torch.exp(0.5 * self.logvar)

    def sample(self, generator=None) -> torch.Tensor:
        eps = torch.randn(self.mean.shape, generator=generator, device=self.mean.device, dtype=self.mean.dtype)
        return self.mean + self.std * eps

    def mode(self):
        return self.mean


class AutoencoderKL(nn.Module):
    def __init__(self, config: VAEConfig):
        super().__init__()
        self.config = config
        self.encoder = Encoder(config)
        self.decoder = Decoder(config)
        lc = config.latent_channels
        self.quant_conv = nn.Conv2d(2 * lc, 2 * lc, 1)
        self.post_quant_conv = nn.Conv2d(lc, lc, 1)
        self.channels_last = False  # unet.to_channels_last

    def _in(self, x):
        return x.contiguous(memory_format=torch.channels_last) if self.channels_last else x

    def encode(self, x: torch.Tensor) -> DiagonalGaussian:
        return DiagonalGaussian(self.encode_moments(x).contiguous())

    def encode_moments(self, x: torch.Tensor) -> torch.Tensor:
        """[B, 2C, h, w] mean / logvar moments in the conv layout (the fused
        training-step noise prep reads them in place: ops/sd_train.py)."""
        return self.quant_conv(self.encoder(self._in(x)))

    def decode(self, z: torch.Tensor) -> torch.Tensor:
        return self.decoder(self.post_quant_conv(self._in(z))).contiguous()


def build_vae(cfg: VAEConfig, device="cpu", dtype=torch.float32, seed: int = 0) -> AutoencoderKL:
    torch.manual_seed(seed)
    return AutoencoderKL(cfg).to(device=device, dtype=dtype)


__all__ = ["VAEConfig", "AutoencoderKL", "build_vae", "L_SCALE_FACTOR", "F"]
