"""UNet2DConditionModel (SD 1.x / 2.x) with diffusers-compatible parameter names.

The SD finetuner / DreamBooth trainer (sd-finetuner-workflow/sd-finetuner/
finetuner.py:648-666, 467-547) and the txt2img predictor
(online-inference/stable-diffusion/service/service.py:163-259) run diffusers'
UNet; this is the same network built on the native ops:

* GroupNorm(+SiLU) -> ``ops.group_norm`` (HIP, fused SiLU in ResNet blocks);
* spatial self-attention and text cross-attention -> ``ops.flash_attention``
  (non-causal; head dims 40/80/160 for SD1.x, 64 for SD2; K/V length 77 for
  the cross attention);
* LayerNorm -> fused LN kernel; convolutions -> MIOpen through torch.

Config keys are read from diffusers' ``unet/config.json``.
"""
from __future__ import annotations

import dataclasses
import json
import math
import os

import torch
import torch.nn as nn
import torch.nn.functional as F

from .. import ops
from ..ops import _lib
from ..ops.conv import conv3x3
from ..ops.linear import SplitKLinear, linear_residual, linear_residual_train, linear_splitk_wgrad
from ..ops.upsample import (phase_gemm_weights, phase_to_dense, phase_weights, upsample_conv_phase,
                           upsample_conv_train, upsample_nearest2x)


@dataclasses.dataclass
class UNetConfig:
    in_channels: int = 4
    out_channels: int = 4
    block_out_channels: tuple = (320, 640, 1280, 1280)
    layers_per_block: int = 2
    cross_attention_dim: int = 768
    attention_head_dim: object = 8          # int (=#heads, diffusers quirk) or per-block list
    down_block_types: tuple = ("CrossAttnDownBlock2D", "CrossAttnDownBlock2D", "CrossAttnDownBlock2D",
                               "DownBlock2D")
    up_block_types: tuple = ("UpBlock2D", "CrossAttnUpBlock2D", "CrossAttnUpBlock2D", "CrossAttnUpBlock2D")
    norm_num_groups: int = 32
    norm_eps: float = 1e-5
    use_linear_projection: bool = False
    flip_sin_to_cos: bool = True
    freq_shift: int = 0
    sample_size: int = 64
    raw: dict = dataclasses.field(default_factory=dict, repr=False)

    @classmethod
    def from_dict(cls, d: dict) -> "UNetConfig":
        kw = {}
        for f in dataclasses.fields(cls):
            if f.name in d and f.name != "raw":
                v = d[f.name]
                kw[f.name] = tuple(v) if isinstance(v, list) else v
        return cls(raw=dict(d), **kw)

    @classmethod
    def from_pretrained(cls, path: str) -> "UNetConfig":
        with open(os.path.join(path, "config.json")) as f:
            return cls.from_dict(json.load(f))

    def to_dict(self) -> dict:
        d = dict(self.raw) if self.raw else {"_class_name": "UNet2DConditionModel"}
        for f in dataclasses.fields(self):
            if f.name != "raw":
                v = getattr(self, f.name)
                d[f.name] = list(v) if isinstance(v, tuple) else v
        return d

    def heads(self, i: int) -> int:
        a = self.attention_head_dim
        return a[i] if isinstance(a, (tuple, list)) else a


def sd15_unet_config() -> UNetConfig:
    return UNetConfig()


def sd2_unet_config(sample_size: int = 96) -> UNetConfig:
    return UNetConfig(cross_attention_dim=1024, attention_head_dim=(5, 10, 20, 20), use_linear_projection=True,
                      sample_size=sample_size)


class GroupNorm(nn.GroupNorm):
    def __init__(self, groups, ch, eps=1e-5, silu=False):
        super().__init__(groups, ch, eps=eps)
        self.silu = silu

    def forward(self, x, add=None):
        return ops.group_norm(x, self.num_groups, self.weight, self.bias, self.eps, silu=self.silu, add=add)


class LayerNorm(nn.LayerNorm):
    def forward(self, x, residual: tuple = ()):
        """``residual`` given: returns (LN(x + sum(residual)), x + sum(residual))
        from one fused kernel (the residual add of the previous sub-block)."""
        return ops.layer_norm(x, self.weight, self.bias, self.eps, residual=residual)


def timestep_embedding(t: torch.Tensor, dim: int, flip_sin_to_cos=True, shift: float = 0.0,
                       max_period: float = 10000.0) -> torch.Tensor:
    """diffusers get_timestep_embedding (K18)."""
    half = dim // 2
    exponent = -math.log(max_period) * torch.arange(half, dtype=torch.float32, device=t.device) / (half - shift)
    emb = t.float()[:, None] * torch.exp(exponent)[None, :]
    emb = torch.cat([torch.sin(emb), torch.cos(emb)], dim=-1)
    if flip_sin_to_cos:
        emb = torch.cat([emb[:, half:], emb[:, :half]], dim=-1)
    if dim % 2:
        emb = F.pad(emb, (0, 1))
    return emb


class TimestepEmbedding(nn.Module):
    def __init__(self, cin, dim):
        super().__init__()
        self.linear_1 = nn.Linear(cin, dim)
        self.linear_2 = nn.Linear(dim, dim)

    def forward(self, x):
        return self.linear_2(F.silu(self.linear_1(x)))


# token-level linears train with split-K weight gradients (ops/linear.py); KCA_SD_SPLITK_WGRAD=0 -> nn.Linear
_Linear = SplitKLinear if os.environ.get("KCA_SD_SPLITK_WGRAD", "1") not in ("0", "false") else nn.Linear


# KCA_SD_FOLD_BIAS=0 keeps the biased convolutions + separate residual add at inference (A/B knob);
# KCA_SD_FOLD_BIAS_TRAIN=0 the same in training
_FOLD_BIAS = os.environ.get("KCA_SD_FOLD_BIAS", "1") not in ("0", "false")
_FOLD_BIAS_TRAIN = os.environ.get("KCA_SD_FOLD_BIAS_TRAIN", "1") not in ("0", "false")


class ResnetBlock2D(nn.Module):
    def __init__(self, cin, cout, temb_ch, groups=32, eps=1e-5):
        super().__init__()
        self.norm1 = GroupNorm(groups, cin, eps, silu=True)
        self.conv1 = nn.Conv2d(cin, cout, 3, padding=1)
        self.time_emb_proj = nn.Linear(temb_ch, cout) if temb_ch else None
        self.norm2 = GroupNorm(groups, cout, eps, silu=True)
        self.dropout = nn.Dropout(0.0)
        self.conv2 = nn.Conv2d(cout, cout, 3, padding=1)
        self.conv_shortcut = nn.Conv2d(cin, cout, 1) if cin != cout else None

    def forward(self, x, temb=None, in_bias=None):
        """``in_bias`` (inference, folded path): a per-channel bias still owed by x's producer (the
        VAE encoder's conv_in): normalised through norm1's add and carried by the residual add."""
        if _FOLD_BIAS and not torch.is_grad_enabled() and x.is_cuda and x.dtype == torch.bfloat16 \
                and x.is_contiguous(memory_format=torch.channels_last) and self.conv1.bias is not None:
            return self._forward_folded(x, temb, in_bias=in_bias)
        if in_bias is not None:
            x = x + in_bias.view(1, -1, 1, 1).to(x.dtype)
        if isinstance(temb, _TembAct):
            return self._forward_act(x, temb.act)
        if isinstance(temb, _TembAdds):
            temb = temb.temb
        if (_FOLD_BIAS_TRAIN and torch.is_grad_enabled() and x.is_cuda and x.dtype == torch.bfloat16
                and x.is_contiguous(memory_format=torch.channels_last) and self.conv1.bias is not None
                and self.conv2.bias is not None):
            return self._forward_folded_train(x, temb)
        h = self.conv1(self.norm1(x))
        t = None
        if self.time_emb_proj is not None and temb is not None:
            t = self.time_emb_proj(F.silu(temb))  # added to h inside norm2 (fused at inference)
        h = self.conv2(self.dropout(self.norm2(h, add=t)))
        sc = self.conv_shortcut(x) if self.conv_shortcut is not None else x
        return sc + h

    def forward_cat(self, x1, x2, temb):
        """Inference on the up-block input ``cat([x1, x2])`` (x1 possibly a _Phased upsampler
        output): norm1 reads both in place and writes the concat once, for the 1x1 shortcut."""
        ph = isinstance(x1, _Phased)
        xn, raw = ops.group_norm_cat(x1.t if ph else x1, x2, self.norm1.num_groups, self.norm1.weight,
                                     self.norm1.bias, self.norm1.eps, silu=True, phase=ph,
                                     x1_add=x1.bias if ph else None)
        return self._forward_folded(raw, temb, xn=xn)

    def _forward_act(self, x, act):
        """Training with the shared silu(temb) (_TembAct)."""
        if (_FOLD_BIAS_TRAIN and x.is_cuda and x.dtype == torch.bfloat16
                and x.is_contiguous(memory_format=torch.channels_last) and self.conv1.bias is not None
                and self.conv2.bias is not None):
            return self._forward_folded_train(x, None, act=act)
        h = self.conv1(self.norm1(x))
        t = self.time_emb_proj(act) if self.time_emb_proj is not None else None
        h = self.conv2(self.dropout(self.norm2(h, add=t)))
        sc = self.conv_shortcut(x) if self.conv_shortcut is not None else x
        return sc + h

    def _forward_folded(self, x, temb, xn=None, in_bias=None):
        """Inference: the convolutions run without bias (MIOpen adds a conv bias in a separate
        broadcast pass over the whole output): conv1's bias joins the time embedding that norm2
        adds inside its statistics, and conv2's (+ the 1x1 shortcut's) bias joins the residual add
        -- one full read+write pass fewer per convolution (profiles/sd_unet_add_attribution_r2.txt)."""
        if in_bias is not None and (xn is not None or self.conv_shortcut is not None):
            x = x + in_bias.view(1, -1, 1, 1).to(x.dtype)  # (the fold below needs the identity shortcut)
            in_bias = None
        if xn is None:
            xn = self.norm1(x) if in_bias is None else \
                self.norm1(x, add=in_bias.float()[None].expand(x.shape[0], -1))
        h = conv3x3(xn, self.conv1.weight)
        add = temb.get(self) if isinstance(temb, _TembAdds) else None  # conv1 bias + time projection, fp32
        if add is None:
            if isinstance(temb, _TembAdds):
                temb = temb.temb
            b1, _ = self._folded_biases()
            add = b1[None].expand(x.shape[0], -1)
            if self.time_emb_proj is not None and temb is not None:
                add = add + self.time_emb_proj(F.silu(temb)).float()
        h = conv3x3(self.norm2(h, add=add), self.conv2.weight)
        _, bias = self._folded_biases()
        if in_bias is not None:
            bias = bias + in_bias.float()
        sc = F.conv2d(x, self.conv_shortcut.weight, None) if self.conv_shortcut is not None else x
        return ops.add_bias_nhwc(sc, h, bias)

    def _forward_folded_train(self, x, temb, act=None):
        """Training with the convolution biases folded out of the convolutions (as at inference):
        conv1's bias joins the [B, C] time embedding the GroupNorm adds, conv2's (+ the shortcut's)
        joins the residual add (ops.add_bias_nhwc_train, bias gradient by a column sum). Exact:
        the same sums in another order; removes each biased convolution's broadcast-add pass and
        PyTorch's bias-gradient reduction over the full activation."""
        h = conv3x3(self.norm1(x), self.conv1.weight)
        add = self.conv1.bias[None].expand(x.shape[0], -1)
        if self.time_emb_proj is not None and (temb is not None or act is not None):
            add = add + self.time_emb_proj(act if act is not None else F.silu(temb))
        h = conv3x3(self.dropout(self.norm2(h, add=add)), self.conv2.weight)
        b2 = None
        if self.conv_shortcut is not None:
            sc = F.conv2d(x, self.conv_shortcut.weight, None)
            b2 = self.conv_shortcut.bias
        else:
            sc = x
        return ops.add_bias2_nhwc_train(sc, h, self.conv2.bias, b2)  # bf16 biases read in the kernel

    def _folded_biases(self):
        """fp32 conv1 bias and conv2 (+ shortcut) bias, cached while the parameters are unchanged
        (one cast/add kernel pair less per block and step)."""
        ps = [p for p in (self.conv1.bias, self.conv2.bias,
                          self.conv_shortcut.bias if self.conv_shortcut is not None else None) if p is not None]
        key = (_WEIGHT_GEN,) + tuple((p.data_ptr(), p._version) for p in ps)
        c = getattr(self, "_fb_cache", None)
        if c is None or c[0] != key:
            b2 = self.conv2.bias.float()
            if self.conv_shortcut is not None and self.conv_shortcut.bias is not None:
                b2 = b2 + self.conv_shortcut.bias.float()
            c = self._fb_cache = (key, self.conv1.bias.float(), b2)
        return c[1], c[2]


class _TembAct:
    """Training: ``silu(temb)`` computed once per UNet forward and shared by every ResNet block's time
    projection -- one SiLU + one SiLU backward per step instead of one pair per block."""

    def __init__(self, act):
        self.act = act


class _TembAdds:
    """Inference: every ResNet block's ``conv1.bias + time_emb_proj(silu(temb))`` (fp32), computed by
    ONE GEMM over the concatenated projection weights (UNet2DConditionModel._temb_adds) instead of
    a SiLU + GEMM + two casts + an add per block; each block's GroupNorm reads its [B, cout] slice
    in place (row stride = the table width)."""

    def __init__(self, temb, table, offsets):
        self.temb, self.table, self.offsets = temb, table, offsets

    def get(self, blk):
        o = self.offsets.get(id(blk))
        return None if o is None else self.table[:, o[0]:o[0] + o[1]]


# Head padding for the self-attention (see Attention.forward); KCA_SD_PAD_HEADS=0
# disables it, KCA_SD_PAD_HEADS_TRAIN=0 only in training. _PAD_GEN counts padded-weight rebuilds so a HIP
# graph captured over the old buffers knows to re-capture (sd_pipeline.UNetGraph).
_TILED_DIMS = (64, 96, 128, 160, 256)  # attention_tiled.hip instantiations (fwd + bwd)
# narrow storage: heads stored 48 wide, staged into the D=64 LDS images of the forward and of both
# backward kernels (attention_tiled.hip StagerNarrow, DS = 48); KCA_SD_NARROW_HEADS=0 pads inference
# heads to 64 (training always runs narrow)
_NARROW = os.environ.get("KCA_SD_NARROW_HEADS", "1") not in ("0", "false")


def padded_head_dim(hd: int, infer: bool = False) -> int:
    """Smallest full-tile head dim >= hd: 40 -> 48 (64 with the narrow path off), 80 -> 96 (160 runs
    natively)."""
    dims = ((48,) if (_NARROW or not infer) else ()) + _TILED_DIMS
    return next((d for d in dims if d >= hd), hd)


_PAD_HEADS = os.environ.get("KCA_SD_PAD_HEADS", "1") not in ("0", "false")
ROWSUM_COL = 40  # SD-1.5's 40-wide heads: padded V column 40 carries ones (softmax row sums on the MFMA)
_ROWSUM = os.environ.get("KCA_SD_ROWSUM_COL", "1") not in ("0", "false")
_PAD_TRAIN = os.environ.get("KCA_SD_PAD_HEADS_TRAIN", "1") not in ("0", "false")
# training: padded heads from one fused QKV GEMM (Attention.forward); KCA_SD_FUSED_QKV_TRAIN=0 keeps the
# three projections + activation pads
_FUSED_QKV_TRAIN = os.environ.get("KCA_SD_FUSED_QKV_TRAIN", "1") not in ("0", "false")
# inference, 48-wide heads: K stored pre-scaled by scale * log2(e) with pad column 40 = 1, so the tiled
# kernel's S MFMAs also subtract the softmax offset (attention_tiled.hip MC); KCA_SD_MAX_COL=0 disables
_MAX_COL = os.environ.get("KCA_SD_MAX_COL", "1") not in ("0", "false")
_PAD_GEN = 0
# Derived-weight caches (folded biases, phase GEMM weights, time-projection and context-K/V tables)
# key on (data_ptr, _version); the native optimizer (kca_adamw) updates parameters in place through
# raw pointers without bumping _version, so the training engine bumps this generation instead
# (UNet2DConditionModel.invalidate_weight_caches, called from TrainEngine._refresh_derived).
_WEIGHT_GEN = 0
# inference: residual adds carried by the preceding GEMM's epilogue (ops.linear_residual);
# KCA_SD_FUSE_RES=0 keeps the separate adds (A/B knob)
_FUSE_RES = os.environ.get("KCA_SD_FUSE_RES", "1") not in ("0", "false")
# inference: upsamplers as im2col + ONE hipBLASLt GEMM of the low-res input with the four 2x2 phase
# kernels (ops/upsample.py: 16 instead of 36 MACs per input pixel, no upsampled activation); the UNet's
# up blocks read that phase layout in place in their concat GroupNorm, the VAE gets it densified.
# KCA_SD_PHASE_UP=0: nearest-x2 (native NHWC kernel) + the 3x3 conv
_PHASE_UP = os.environ.get("KCA_SD_PHASE_UP", "1") not in ("0", "false")
# training: the same phase GEMM with its backward (ops/upsample.py upsample_conv_train); KCA_SD_PHASE_UP_TRAIN=0
# keeps nearest-x2 + the 3x3 convolution
_PHASE_UP_TRAIN = os.environ.get("KCA_SD_PHASE_UP_TRAIN", "1") not in ("0", "false")
# inference: the up blocks' GroupNorm reads [x | skip] in place and writes the concat once for the
# 1x1 shortcut (ops.group_norm_cat) instead of torch.cat + GroupNorm; KCA_SD_CAT_GN=0 disables
_CAT_GN = os.environ.get("KCA_SD_CAT_GN", "1") not in ("0", "false")
# inference: all ResNet time projections as one GEMM (_TembAdds); KCA_SD_TEMB_BATCH=0 disables
_TEMB_BATCH = os.environ.get("KCA_SD_TEMB_BATCH", "1") not in ("0", "false")


def pad_generation() -> int:
    return _PAD_GEN


class Attention(nn.Module):
    """diffusers Attention (to_q/to_k/to_v/to_out.0) over [B, S, C] tokens."""

    def __init__(self, dim, heads, head_dim, cross_dim=None, bias_qkv=False):
        super().__init__()
        inner = heads * head_dim
        self.heads = heads
        self.to_q = _Linear(dim, inner, bias=bias_qkv)
        self.to_k = _Linear(cross_dim or dim, inner, bias=bias_qkv)
        self.to_v = _Linear(cross_dim or dim, inner, bias=bias_qkv)
        self.to_out = nn.ModuleList([_Linear(inner, dim), nn.Dropout(0.0)])
        self.cross = cross_dim is not None
        self._padded = None

    def train(self, mode: bool = True):
        self._padded = None  # weights may change while training: rebuild on the next inference call
        return super().train(mode)

    def _padded_weights(self, hd: int, dp: int, max_col: bool = False):
        """One fused QKV weight with each head zero-padded to dp rows, and the
        out-projection with matching zero columns (built once per eval phase;
        ``train()`` drops it). ``max_col``: K rows pre-scaled by scale * log2(e), K column 40 = 1."""
        p = getattr(self, "_padded", None)
        if p is not None and p[3] != max_col:
            p = None
        if p is None:
            global _PAD_GEN
            H = self.heads
            C = self.to_q.weight.shape[1]
            w = self.to_q.weight.new_zeros(3, H, dp, C)
            b = self.to_q.weight.new_zeros(3, H, dp)
            for i, lin in enumerate((self.to_q, self.to_k, self.to_v)):
                w[i, :, :hd] = lin.weight.view(H, hd, C)
                if lin.bias is not None:
                    b[i, :, :hd] = lin.bias.view(H, hd)
            has_b = any(lin.bias is not None for lin in (self.to_q, self.to_k, self.to_v))
            if dp in (48, 64) and hd == ROWSUM_COL:
                # V column 40 = 1 for every key (zero weights + unit bias): the D=64-image attention
                # kernel reads the softmax row sums off O's column 40 (ops.flash_attention
                # rowsum_col); the out-projection's zero columns ignore it
                b[2, :, ROWSUM_COL] = 1.0
                has_b = True
            if max_col:  # softmax scale and log2(e) folded into K (fp32 product, one bf16 rounding)
                f = math.log2(math.e) / math.sqrt(hd)
                for i_, lin in ((1, self.to_k),):
                    w[i_, :, :hd] = (lin.weight.float().view(H, hd, C) * f).to(w.dtype)
                    if lin.bias is not None:
                        b[i_, :, :hd] = (lin.bias.float().view(H, hd) * f).to(b.dtype)
                b[1, :, ROWSUM_COL] = 1.0
            wo = self.to_out[0].weight
            wo_p = wo.new_zeros(wo.shape[0], H, dp)
            wo_p[:, :, :hd] = wo.view(wo.shape[0], H, hd)
            p = self._padded = (w.view(3 * H * dp, C), b.view(-1) if has_b else None, wo_p.view(wo.shape[0], H * dp),
                                max_col)
            _PAD_GEN += 1
        return p[:3]

    def forward(self, x, ctx=None):
        B, S, _ = x.shape
        hd = self.to_q.weight.shape[0] // self.heads
        train = torch.is_grad_enabled()
        dpad = padded_head_dim(hd, infer=not train)
        pad = ctx is None and x.is_cuda and dpad != hd and hd % 8 == 0 and S % 128 == 0 and _PAD_HEADS
        if pad and train and _PAD_TRAIN and _FUSED_QKV_TRAIN:
            # training: ONE GEMM with the zero-padded q/k/v weights (built per step from the three
            # Linears, differentiably: the weight gradients slice back through F.pad / cat) writes the
            # padded heads straight into a fused [B, S, 3*H*dpad] buffer; the attention backward writes
            # dQ/dK/dV into one buffer (ops.qkv_rope_attention); the out-projection takes the padded
            # heads through zero weight columns -- no activation pads, slices or per-projection grad adds
            H, C = self.heads, x.shape[-1]

            def _padw(lin):
                return F.pad(lin.weight.view(H, hd, C), (0, 0, 0, dpad - hd)).reshape(H * dpad, C)

            w = torch.cat([_padw(self.to_q), _padw(self.to_k), _padw(self.to_v)])
            bs = [lin.bias for lin in (self.to_q, self.to_k, self.to_v)]
            b = None
            if any(t is not None for t in bs):
                b = torch.cat([F.pad((t if t is not None else w.new_zeros(H * hd)).view(H, hd), (0, dpad - hd))
                               .reshape(-1) for t in bs])
            qkv = linear_splitk_wgrad(x, w, b)
            o = ops.qkv_rope_attention(qkv, H, dpad, 0, False, causal=False, scale=1.0 / math.sqrt(hd))
            wo = self.to_out[0].weight
            wo_p = F.pad(wo.view(wo.shape[0], H, hd), (0, dpad - hd)).reshape(wo.shape[0], H * dpad)
            return linear_splitk_wgrad(o, wo_p, self.to_out[0].bias)
        if pad and train and _PAD_TRAIN:
            # training: pad the q/k/v activations instead (F.pad's backward slices the
            # gradients back) so the backward also runs the full-tile D=64 kernels.
            # Attention fwd+bwd 4.50 -> 3.31 ms; DreamBooth 93.4 -> 96.4 samples/s
            # (same-box A/B, profiles/sd_bench_r1_v11_gn_add_padtrain.jsonl);
            # KCA_SD_PAD_HEADS_TRAIN=0 disables.
            dp = dpad - hd
            q, k, v = (F.pad(lin(x).view(B, S, self.heads, hd), (0, dp))
                       for lin in (self.to_q, self.to_k, self.to_v))
            o = ops.flash_attention(q, k, v, causal=False, scale=1.0 / math.sqrt(hd))
            return self.to_out[0](o[..., :hd].reshape(B, S, -1))
        if pad and not train:
            # inference self-attention on the full-tile kernels (attention_tiled.hip: the 40-wide
            # heads stored 48 wide in a D=64 LDS image, the 80-wide ones padded to 96): zero q/k
            # columns leave Q.K^T unchanged, zero v columns give zero outputs that meet zero
            # out-projection columns. SD-1.5 64x64-latent self-attention (B16 H8 S4096 d40)
            # 1.04 -> 0.71 ms on MI355X at 64 wide (profiles/attn_bench_r1_v7_d64.jsonl).
            rs = dpad in (48, 64) and hd == ROWSUM_COL and _ROWSUM
            mc = rs and dpad == 48 and _MAX_COL
            w, b, wo = self._padded_weights(hd, dpad, max_col=mc)
            qkv = F.linear(x, w, b).view(B, S, 3, self.heads, dpad)
            o = ops.flash_attention(qkv[:, :, 0], qkv[:, :, 1], qkv[:, :, 2], causal=False,
                                    scale=math.log(2.0) if mc else 1.0 / math.sqrt(hd),
                                    rowsum_col=ROWSUM_COL if rs else -1, max_col=ROWSUM_COL if mc else -1)
            return F.linear(o.reshape(B, S, -1), wo, self.to_out[0].bias)
        kv = ctx.get(self) if isinstance(ctx, CtxKV) else None
        if kv is not None:  # text K/V precomputed once per prompt batch (UNet2DConditionModel.ctx_kv)
            q = self.to_q(x)
            k, v = kv
        else:
            c = x if ctx is None else (ctx.ctx if isinstance(ctx, CtxKV) else ctx)
            q = self.to_q(x)
            k = self.to_k(c)
            v = self.to_v(c)
        hd = q.shape[-1] // self.heads
        L = k.shape[1]
        o = ops.flash_attention(q.view(B, S, self.heads, hd), k.view(B, L, self.heads, hd),
                                v.view(B, L, self.heads, hd), causal=False)
        return self.to_out[0](o.reshape(B, S, -1))


class CtxKV:
    """Inference: the text context's K and V for every cross-attention layer, from ONE GEMM over
    the concatenated to_k / to_v weights (UNet2DConditionModel.ctx_kv). The context is fixed for
    all denoising steps of a prompt batch, so the 50-step loop
    (online-inference/stable-diffusion/service/service.py:244-252) computes these projections once
    instead of 2 x 16 GEMMs per step; each layer reads its K / V slices of ``table`` [B, L, width]
    in place (row stride = width)."""

    def __init__(self, ctx, table, offsets):
        self.ctx, self.table, self.offsets = ctx, table, offsets

    def get(self, attn):
        o = self.offsets.get(id(attn))
        if o is None:
            return None
        ko, vo, n = o
        return self.table[:, :, ko:ko + n], self.table[:, :, vo:vo + n]


class GEGLU(nn.Module):
    def __init__(self, dim, inner):
        super().__init__()
        self.proj = _Linear(dim, inner * 2)

    def forward(self, x):
        return ops.geglu(self.proj(x))


class FeedForward(nn.Module):
    def __init__(self, dim, mult=4):
        super().__init__()
        inner = dim * mult
        self.net = nn.ModuleList([GEGLU(dim, inner), nn.Dropout(0.0), _Linear(inner, dim)])

    def forward(self, x):
        return self.net[2](self.net[0](x))


class BasicTransformerBlock(nn.Module):
    def __init__(self, dim, heads, head_dim, cross_dim):
        super().__init__()
        self.norm1 = LayerNorm(dim)
        self.attn1 = Attention(dim, heads, head_dim)
        self.norm2 = LayerNorm(dim)
        self.attn2 = Attention(dim, heads, head_dim, cross_dim)
        self.norm3 = LayerNorm(dim)
        self.ff = FeedForward(dim)

    def forward(self, x, ctx):
        # the residual adds after attn1 / attn2 ride in the next LayerNorm kernel
        n2, x = self.norm2(self.attn1(self.norm1(x)), residual=(x,))
        n3, x = self.norm3(self.attn2(n2, ctx), residual=(x,))
        if _FUSE_RES:  # FF out-projection + bias + residual: one GEMM (training: with its own backward)
            out = self.ff.net[2]
            return linear_residual_train(self.ff.net[0](n3), out.weight, out.bias, x)
        return x + self.ff(n3)


class Transformer2DModel(nn.Module):
    def __init__(self, ch, heads, cross_dim, groups=32, linear_proj=False):
        super().__init__()
        self.norm = nn.GroupNorm(groups, ch, eps=1e-6)
        self.linear_proj = linear_proj
        self.proj_in = _Linear(ch, ch) if linear_proj else nn.Conv2d(ch, ch, 1)
        self.transformer_blocks = nn.ModuleList([BasicTransformerBlock(ch, heads, ch // heads, cross_dim)])
        self.proj_out = _Linear(ch, ch) if linear_proj else nn.Conv2d(ch, ch, 1)

    def forward(self, x, ctx):
        B, C, H, W = x.shape
        res = x
        h = ops.group_norm(x, self.norm.num_groups, self.norm.weight, self.norm.bias, self.norm.eps)
        if _is_cl(h):
            # channels-last: the [B, HW, C] token view is free and the 1x1 proj
            # convs are plain GEMMs on it
            t = h.permute(0, 2, 3, 1).reshape(B, H * W, C)
            t = _proj(self.proj_in, t)
            for blk in self.transformer_blocks:
                t = blk(t, ctx)
            if _FUSE_RES:  # proj_out + bias + residual: one GEMM (training: with its own backward)
                w = self.proj_out.weight
                o = linear_residual_train(t, w.reshape(w.shape[0], w.shape[1]), self.proj_out.bias,
                                          res.permute(0, 2, 3, 1))
                return o.permute(0, 3, 1, 2)
            t = _proj(self.proj_out, t)
            return t.view(B, H, W, C).permute(0, 3, 1, 2) + res
        if self.linear_proj:
            h = self.proj_in(h.permute(0, 2, 3, 1).reshape(B, H * W, C))
        else:
            h = self.proj_in(h).permute(0, 2, 3, 1).reshape(B, H * W, C)
        for blk in self.transformer_blocks:
            h = blk(h, ctx)
        if self.linear_proj:
            h = self.proj_out(h).reshape(B, H, W, C).permute(0, 3, 1, 2)
        else:
            h = self.proj_out(h.reshape(B, H, W, C).permute(0, 3, 1, 2).contiguous())
        return h + res


def _is_cl(x: torch.Tensor) -> bool:
    return x.dim() == 4 and x.is_contiguous(memory_format=torch.channels_last) and not x.is_contiguous()


def _proj(m: nn.Module, t: torch.Tensor) -> torch.Tensor:
    """nn.Linear, or a 1x1 nn.Conv2d applied as the same GEMM on a token view."""
    if isinstance(m, nn.Linear):
        return m(t)
    return linear_splitk_wgrad(t, m.weight.reshape(m.weight.shape[0], m.weight.shape[1]), m.bias)


def to_channels_last(model: nn.Module, weights: bool = True) -> nn.Module:
    """Run a UNet / VAE channels-last end to end on MI355X: NHWC activations
    (MIOpen's NHWC convolutions without per-call layout transposes, NHWC
    GroupNorm kernels, free token views for attention). ``weights`` also
    converts the conv weights; the training engine keeps that order in its
    flat buffer (train/engine.py)."""
    from ..utils import miopen, tunable
    miopen.configure()
    if next(model.parameters()).is_cuda:
        tunable.ensure(tunable.SD_FILE)  # MI355X-tuned hipBLASLt choices for the SD GEMM shapes
    model.channels_last = True
    if weights:
        model.to(memory_format=torch.channels_last)
    return model


class Downsample2D(nn.Module):
    def __init__(self, ch, pad=1):
        super().__init__()
        self.conv = nn.Conv2d(ch, ch, 3, stride=2, padding=pad)
        self.asym = pad == 0

    def forward(self, x):
        if self.asym:
            cl = _is_cl(x)
            if cl and _lib.use_native(x) and not (torch.is_grad_enabled() and x.requires_grad) \
                    and x.shape[1] % 8 == 0 and x.data_ptr() % 16 == 0:
                # channels-last pad in one pass (F.pad leaves channels-last: fill + transposing copy +
                # the copy back, ~1.3 ms at 16 x 128 x 512^2 in the DreamBooth step's VAE encode)
                N, C, H, W = x.shape
                out = torch.empty(N, C, H + 1, W + 1, device=x.device, dtype=x.dtype,
                                  memory_format=torch.channels_last)
                _lib.call("kca_pad_br_nhwc", x.data_ptr(), out.data_ptr(), N, H, W, C, _lib.stream())
                x = out
            else:
                x = F.pad(x, (0, 1, 0, 1))
                if cl:
                    x = x.contiguous(memory_format=torch.channels_last)
        return self.conv(x)


class Upsample2D(nn.Module):
    def __init__(self, ch):
        super().__init__()
        self.conv = nn.Conv2d(ch, ch, 3, padding=1)
        self.phase_out = False  # set by the UNet: its up blocks read the phase layout in place

    def _gemm_weights(self):
        cw = self.conv.weight
        key = (_WEIGHT_GEN, cw.data_ptr(), cw._version)
        c = getattr(self, "_phase_cache", None)
        if c is None or c[0] != key:  # re-derived when the conv weight is replaced or updated
            c = self._phase_cache = (key, phase_gemm_weights(cw))
        return c[1]

    def forward(self, x):
        infer = (not torch.is_grad_enabled() and x.is_cuda and x.dtype == torch.bfloat16 and _is_cl(x)
                 and x.shape[1] % 8 == 0)
        if infer and _PHASE_UP:
            t = upsample_conv_phase(x, self._gemm_weights())
            hw = (x.shape[2] * 2, x.shape[3] * 2)
            if self.phase_out:
                return _Phased(t, self.conv.bias, hw)
            return phase_to_dense(t, hw, self.conv.bias)
        if infer:
            return self.conv(upsample_nearest2x(x))
        if _PHASE_UP_TRAIN and torch.is_grad_enabled() and x.is_cuda and x.dtype == torch.bfloat16 and _is_cl(x):
            return upsample_conv_train(x, self.conv.weight, self.conv.bias)
        return self.conv(F.interpolate(x, scale_factor=2.0, mode="nearest"))


class _Phased:
    """An upsampler output left in the 2x2 phase layout (inference): ``t`` [N, 4C, H/2+1, W/2+1]
    channels-last without the conv bias; the next up-block's concat GroupNorm reads it in place.
    ``dense()`` materialises it (+ bias) with the native scatter kernel (fallback)."""

    def __init__(self, t, bias, hw):
        self.t, self.bias, self.hw = t, bias, hw

    def dense(self):
        return phase_to_dense(self.t, self.hw, self.bias)


class DownBlock(nn.Module):
    def __init__(self, cin, cout, temb, n, attn: bool, heads, cross_dim, add_down, groups, eps, linear_proj):
        super().__init__()
        self.resnets = nn.ModuleList([ResnetBlock2D(cin if i == 0 else cout, cout, temb, groups, eps)
                                      for i in range(n)])
        self.attentions = nn.ModuleList([Transformer2DModel(cout, heads, cross_dim, groups, linear_proj)
                                         for _ in range(n)]) if attn else None
        self.downsamplers = nn.ModuleList([Downsample2D(cout)]) if add_down else None

    def forward(self, x, temb, ctx):
        skips = []
        for i, r in enumerate(self.resnets):
            x = r(x, temb)
            if self.attentions is not None:
                x = self.attentions[i](x, ctx)
            skips.append(x)
        if self.downsamplers is not None:
            x = self.downsamplers[0](x)
            skips.append(x)
        return x, skips


class UpBlock(nn.Module):
    def __init__(self, cin, cout, prev, temb, n, attn, heads, cross_dim, add_up, groups, eps, linear_proj):
        super().__init__()
        rs = []
        for i in range(n):
            skip = cin if i == n - 1 else cout
            rin = prev if i == 0 else cout
            rs.append(ResnetBlock2D(rin + skip, cout, temb, groups, eps))
        self.resnets = nn.ModuleList(rs)
        self.attentions = nn.ModuleList([Transformer2DModel(cout, heads, cross_dim, groups, linear_proj)
                                         for _ in range(n)]) if attn else None
        self.upsamplers = nn.ModuleList([Upsample2D(cout)]) if add_up else None

    def forward(self, x, skips, temb, ctx):
        for i, r in enumerate(self.resnets):
            skip = skips.pop()
            if (_CAT_GN and not torch.is_grad_enabled() and skip.is_cuda and _is_cl(skip) and _FOLD_BIAS
                    and r.conv1.bias is not None and (isinstance(x, _Phased) or _is_cl(x))):
                x = r.forward_cat(x, skip, temb)
            else:
                x = r(torch.cat([x.dense() if isinstance(x, _Phased) else x, skip], dim=1), temb)
            if self.attentions is not None:
                x = self.attentions[i](x, ctx)
        if self.upsamplers is not None:
            x = self.upsamplers[0](x)
        return x


class MidBlock(nn.Module):
    def __init__(self, ch, temb, heads, cross_dim, groups, eps, linear_proj):
        super().__init__()
        self.attentions = nn.ModuleList([Transformer2DModel(ch, heads, cross_dim, groups, linear_proj)])
        self.resnets = nn.ModuleList([ResnetBlock2D(ch, ch, temb, groups, eps), ResnetBlock2D(ch, ch, temb, groups, eps)])

    def forward(self, x, temb, ctx):
        x = self.resnets[0](x, temb)
        x = self.attentions[0](x, ctx)
        return self.resnets[1](x, temb)


class UNet2DConditionModel(nn.Module):
    def __init__(self, config: UNetConfig):
        super().__init__()
        c = config
        self.config = c
        ch = c.block_out_channels
        temb = ch[0] * 4
        g, eps = c.norm_num_groups, c.norm_eps
        self.conv_in = nn.Conv2d(c.in_channels, ch[0], 3, padding=1)
        self.time_embedding = TimestepEmbedding(ch[0], temb)
        downs = []
        out = ch[0]
        for i, kind in enumerate(c.down_block_types):
            cin, out = out, ch[i]
            downs.append(DownBlock(cin, out, temb, c.layers_per_block, kind.startswith("CrossAttn"), c.heads(i),
                                   c.cross_attention_dim, i < len(ch) - 1, g, eps, c.use_linear_projection))
        self.down_blocks = nn.ModuleList(downs)
        self.mid_block = MidBlock(ch[-1], temb, c.heads(len(ch) - 1), c.cross_attention_dim, g, eps,
                                  c.use_linear_projection)
        rch = list(reversed(ch))
        rheads = [c.heads(i) for i in reversed(range(len(ch)))]
        ups = []
        prev = rch[0]
        for i, kind in enumerate(c.up_block_types):
            out = rch[i]
            cin = rch[min(i + 1, len(ch) - 1)]
            ups.append(UpBlock(cin, out, prev, temb, c.layers_per_block + 1, kind.startswith("CrossAttn"),
                               rheads[i], c.cross_attention_dim, i < len(ch) - 1, g, eps,
                               c.use_linear_projection))
            prev = out
        self.up_blocks = nn.ModuleList(ups)
        for blk in self.up_blocks:  # every up-block upsampler feeds the next block's concat GroupNorm
            if blk.upsamplers is not None:
                blk.upsamplers[0].phase_out = True
        self.conv_norm_out = GroupNorm(g, ch[0], eps, silu=True)
        self.conv_out = nn.Conv2d(ch[0], c.out_channels, 3, padding=1)
        self.gradient_checkpointing = False
        self.channels_last = False

    def enable_gradient_checkpointing(self, on: bool = True):
        self.gradient_checkpointing = on

    def invalidate_weight_caches(self):
        """Parameters changed in place: every derived-weight cache rebuilds on next use."""
        global _WEIGHT_GEN
        _WEIGHT_GEN += 1
        for m in self.modules():
            if isinstance(m, Attention):
                m._padded = None

    def _temb_adds(self, temb: torch.Tensor) -> _TembAdds:
        """One GEMM for every ResNet block's time projection (+ its conv1 bias, fp32): see _TembAdds."""
        rs = [m for m in self.modules() if isinstance(m, ResnetBlock2D) and m.time_emb_proj is not None
              and m.conv1.bias is not None]
        ps = [p for r in rs for p in (r.time_emb_proj.weight, r.time_emb_proj.bias, r.conv1.bias) if p is not None]
        key = (_WEIGHT_GEN,) + tuple((p.data_ptr(), p._version) for p in ps)
        c = getattr(self, "_temb_cache", None)
        if c is None or c[0] != key:
            w = torch.cat([r.time_emb_proj.weight for r in rs])
            b = torch.cat([r.conv1.bias.float() + (r.time_emb_proj.bias.float() if r.time_emb_proj.bias is not None
                                                   else 0.0) for r in rs])
            offs, o = {}, 0
            for r in rs:
                n = r.time_emb_proj.weight.shape[0]
                offs[id(r)] = (o, n)
                o += n
            c = self._temb_cache = (key, w, b, offs)
        _, w, b, offs = c
        return _TembAdds(temb, torch.add(b, F.linear(F.silu(temb), w)), offs)

    def ctx_kv(self, ctx: torch.Tensor, out: CtxKV | None = None) -> CtxKV:
        """Every cross-attention layer's K and V of the text context ``ctx`` [B, L, cross_dim] as one
        GEMM (see CtxKV). ``out``: recompute into that object's table (static graph buffers)."""
        attns = [m for m in self.modules() if isinstance(m, Attention) and m.cross]
        ps = [p for a in attns for p in (a.to_k.weight, a.to_v.weight, a.to_k.bias, a.to_v.bias) if p is not None]
        key = (_WEIGHT_GEN,) + tuple((p.data_ptr(), p._version) for p in ps)
        c = getattr(self, "_ctxkv_cache", None)
        if c is None or c[0] != key:
            ws, bs, offs, o = [], [], {}, 0
            for a in attns:
                n = a.to_k.weight.shape[0]
                offs[id(a)] = (o, o + n, n)
                o += 2 * n
                for lin in (a.to_k, a.to_v):
                    ws.append(lin.weight)
                    bs.append(lin.bias if lin.bias is not None else lin.weight.new_zeros(n))
            has_b = any(lin.bias is not None for a in attns for lin in (a.to_k, a.to_v))
            c = self._ctxkv_cache = (key, torch.cat(ws), torch.cat(bs) if has_b else None, offs)
        _, w, b, offs = c
        ctx = ctx.to(w.dtype)
        if out is not None and out.table.shape[:2] == ctx.shape[:2] and out.table.shape[2] == w.shape[0]:
            out.table.copy_(F.linear(ctx, w, b))
            out.ctx = ctx
            return out
        return CtxKV(ctx, F.linear(ctx, w, b), offs)

    def _run(self, fn, *args):
        if self.gradient_checkpointing and self.training and torch.is_grad_enabled():
            from torch.utils.checkpoint import checkpoint
            return checkpoint(fn, *args, use_reentrant=False)
        return fn(*args)

    def forward(self, sample: torch.Tensor, timestep, encoder_hidden_states: torch.Tensor):
        c = self.config
        if not torch.is_tensor(timestep):
            timestep = torch.tensor([timestep], device=sample.device)
        t = timestep.to(sample.device).reshape(-1).expand(sample.shape[0])
        temb = timestep_embedding(t, c.block_out_channels[0], c.flip_sin_to_cos, c.freq_shift).to(sample.dtype)
        temb = self.time_embedding(temb)
        if (_TEMB_BATCH and _FOLD_BIAS and not torch.is_grad_enabled() and self.channels_last and temb.is_cuda
                and temb.dtype == torch.bfloat16):
            temb = self._temb_adds(temb)
        elif torch.is_grad_enabled() and temb.is_cuda and not self.gradient_checkpointing:
            temb = _TembAct(F.silu(temb))
        ctx = encoder_hidden_states if isinstance(encoder_hidden_states, CtxKV) else \
            encoder_hidden_states.to(sample.dtype)
        if self.channels_last:
            sample = sample.contiguous(memory_format=torch.channels_last)
        x = self.conv_in(sample)
        skips = [x]
        for blk in self.down_blocks:
            x, s = self._run(blk, x, temb, ctx)
            skips.extend(s)
        x = self._run(self.mid_block, x, temb, ctx)
        for blk in self.up_blocks:
            n = len(blk.resnets)
            mine = skips[-n:]
            del skips[-n:]
            x = self._run(lambda a, b, cc, *sk, _blk=blk: _blk(a, list(sk), b, cc), x, temb, ctx, *mine)
        if isinstance(x, _Phased):  # a config whose last up block upsamples
            x = x.dense()
        return self.conv_out(self.conv_norm_out(x)).contiguous()


def build_unet(cfg: UNetConfig, device="cpu", dtype=torch.float32, seed: int = 0) -> UNet2DConditionModel:
    torch.manual_seed(seed)
    m = UNet2DConditionModel(cfg)
    return m.to(device=device, dtype=dtype)
