"""CLIP text encoder (K23): the frozen conditioning model of SD 1.x / 2.x.

Parameter names follow transformers' ``CLIPTextModel`` (``text_model.*``) so a
diffusers pipeline's ``text_encoder/`` loads unchanged (sd-finetuner/
finetuner.py:648-659 loads it with CLIPTextModel.from_pretrained). Attention
runs through the native flash kernel (causal, head_dim 64), LayerNorms through
the fused LN kernel.
"""
from __future__ import annotations

import dataclasses
import json
import os

import torch
import torch.nn as nn
import torch.nn.functional as F

from .. import ops


@dataclasses.dataclass
class CLIPTextConfig:
    vocab_size: int = 49408
    hidden_size: int = 768
    intermediate_size: int = 3072
    num_hidden_layers: int = 12
    num_attention_heads: int = 12
    max_position_embeddings: int = 77
    hidden_act: str = "quick_gelu"
    layer_norm_eps: float = 1e-5
    eos_token_id: int = 49407
    raw: dict = dataclasses.field(default_factory=dict, repr=False)

    @classmethod
    def from_dict(cls, d: dict) -> "CLIPTextConfig":
        d = d.get("text_config", d)
        kw = {f.name: d[f.name] for f in dataclasses.fields(cls) if f.name in d and f.name != "raw"}
        return cls(raw=dict(d), **kw)

    @classmethod
    def from_pretrained(cls, path: str) -> "CLIPTextConfig":
        with open(os.path.join(path, "config.json")) as f:
            return cls.from_dict(json.load(f))

    def to_dict(self) -> dict:
        d = dict(self.raw) if self.raw else {"model_type": "clip_text_model",
                                             "architectures": ["CLIPTextModel"]}
        d.update({f.name: getattr(self, f.name) for f in dataclasses.fields(self) if f.name != "raw"})
        return d


class _LN(nn.LayerNorm):
    def forward(self, x, residual=()):
        return ops.layer_norm(x, self.weight, self.bias, self.eps, residual=residual)


class CLIPAttention(nn.Module):
    def __init__(self, c: CLIPTextConfig):
        super().__init__()
        d = c.hidden_size
        self.h = c.num_attention_heads
        self.q_proj = nn.Linear(d, d)
        self.k_proj = nn.Linear(d, d)
        self.v_proj = nn.Linear(d, d)
        self.out_proj = nn.Linear(d, d)

    def forward(self, x, causal=True, kv_len=None):
        B, S, d = x.shape
        hd = d // self.h
        q = self.q_proj(x).view(B, S, self.h, hd)
        k = self.k_proj(x).view(B, S, self.h, hd)
        v = self.v_proj(x).view(B, S, self.h, hd)
        o = ops.flash_attention(q, k, v, causal=causal, kv_len=kv_len)
        return self.out_proj(o.reshape(B, S, d))


class CLIPMLP(nn.Module):
    def __init__(self, c: CLIPTextConfig):
        super().__init__()
        self.fc1 = nn.Linear(c.hidden_size, c.intermediate_size)
        self.fc2 = nn.Linear(c.intermediate_size, c.hidden_size)
        self.act = c.hidden_act

    def forward(self, x):
        h = self.fc1(x)
        if self.act == "quick_gelu":
            h = ops.quick_gelu(h)
        elif self.act in ("gelu_new", "gelu_pytorch_tanh"):
            h = ops.gelu(h, "tanh")
        else:
            h = ops.gelu(h, "none")
        return self.fc2(h)


class CLIPEncoderLayer(nn.Module):
    def __init__(self, c: CLIPTextConfig):
        super().__init__()
        self.self_attn = CLIPAttention(c)
        self.layer_norm1 = _LN(c.hidden_size, eps=c.layer_norm_eps)
        self.mlp = CLIPMLP(c)
        self.layer_norm2 = _LN(c.hidden_size, eps=c.layer_norm_eps)

    def forward(self, h, kv_len=None):
        a = self.self_attn(self.layer_norm1(h), True, kv_len)
        x2, h = self.layer_norm2(h, residual=(a,))
        return h + self.mlp(x2)


class _Embeddings(nn.Module):
    def __init__(self, c: CLIPTextConfig):
        super().__init__()
        self.token_embedding = nn.Embedding(c.vocab_size, c.hidden_size)
        self.position_embedding = nn.Embedding(c.max_position_embeddings, c.hidden_size)


class _Encoder(nn.Module):
    def __init__(self, c: CLIPTextConfig):
        super().__init__()
        self.layers = nn.ModuleList([CLIPEncoderLayer(c) for _ in range(c.num_hidden_layers)])


class _TextTransformer(nn.Module):
    def __init__(self, c: CLIPTextConfig):
        super().__init__()
        self.embeddings = _Embeddings(c)
        self.encoder = _Encoder(c)
        self.final_layer_norm = _LN(c.hidden_size, eps=c.layer_norm_eps)


class CLIPTextModel(nn.Module):
    def __init__(self, config: CLIPTextConfig):
        super().__init__()
        self.config = config
        self.text_model = _TextTransformer(config)

    def forward(self, input_ids: torch.Tensor, attention_mask: torch.Tensor | None = None,
                output_hidden_states: bool = False):
        tm = self.text_model
        S = input_ids.shape[1]
        h = tm.embeddings.token_embedding(input_ids) + tm.embeddings.position_embedding(
            torch.arange(S, device=input_ids.device))
        kv_len = None
        if attention_mask is not None and not bool(attention_mask.all()):
            kv_len = attention_mask.sum(-1).to(torch.int32)
        hidden = [h]
        for layer in tm.encoder.layers:
            h = layer(h, kv_len)
            hidden.append(h)
        last = tm.final_layer_norm(h)
        if output_hidden_states:
            return last, hidden
        return last

    def pooled(self, last: torch.Tensor, input_ids: torch.Tensor) -> torch.Tensor:
        """EOS-token pooled output (transformers' pooler_output)."""
        idx = (input_ids == self.config.eos_token_id).int().argmax(-1)
        return last[torch.arange(last.shape[0], device=last.device), idx]

    @classmethod
    def from_pretrained(cls, path: str, device="cpu", dtype=torch.float32):
        from ..io.hf import read_hf_state_dict
        cfg = CLIPTextConfig.from_pretrained(path)
        with torch.device("meta"):
            m = cls(cfg)
        m = m.to_empty(device=device).to(dtype)
        m.load_hf(read_hf_state_dict(path))
        return m

    def load_hf(self, sd: dict):
        """Load a transformers CLIPTextModel state dict (with or without the
        ``text_model.`` prefix; transformers 5 drops it in memory)."""
        out = {}
        for k, v in sd.items():
            if k.endswith("position_ids"):
                continue
            out[k if k.startswith("text_model.") else "text_model." + k] = v
        dt = next(self.parameters()).dtype
        self.load_state_dict({k: v.to(dt) for k, v in out.items()}, strict=True)

    def save_pretrained(self, path: str):
        from safetensors.torch import save_file
        os.makedirs(path, exist_ok=True)
        with open(os.path.join(path, "config.json"), "w") as f:
            json.dump(self.config.to_dict(), f, indent=2)
        save_file({k: v.contiguous().cpu() for k, v in self.state_dict().items()},
                  os.path.join(path, "model.safetensors"), metadata={"format": "pt"})


def build_clip_text(cfg: CLIPTextConfig, device="cpu", dtype=torch.float32, seed: int = 0) -> CLIPTextModel:
    g = torch.Generator().manual_seed(seed)
    m = CLIPTextModel(cfg)
    with torch.no_grad():
        for n, p in m.named_parameters():
            if p.dim() >= 2:
                p.copy_(torch.randn(p.shape, generator=g) * 0.02)
            elif n.endswith("weight"):
                p.fill_(1.0)
            else:
                p.zero_()
    return m.to(device=device, dtype=dtype)


__all__ = ["CLIPTextConfig", "CLIPTextModel", "build_clip_text", "F"]
