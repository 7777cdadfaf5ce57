"""HF <-> native parameter-name mapping for the causal-LM family.

The finetuner must read the same model directories the reference's HF
``from_pretrained`` reads (finetuner-workflow/finetuner/finetuner.py:816-824)
and write ``checkpoint-N`` / ``final`` directories the reference's serving side
(``inference.py`` pipeline, ``finetune-workflow.yaml:583-619``) can load back.

Native layout differences handled here:
* Q/K/V are ONE fused [3*d, d] weight (rows ordered q|k|v, each [H, D]);
  GPT-J has three bias-free projections, GPT-2 a Conv1D ``c_attn`` ([d, 3d],
  transposed), NeoX/BLOOM an interleaved ``query_key_value`` ([H, 3, D] rows).
* GPT-2 Conv1D weights are stored [in, out] and transposed on the way in/out.
"""
from __future__ import annotations

import re

import torch

from .config import LMConfig


def _neox_qkv_to_native(w: torch.Tensor, H: int, D: int) -> torch.Tensor:
    # HF rows: [H, 3, D]  ->  native rows: [3, H, D]
    shp = w.shape
    w = w.view(H, 3, D, *shp[1:]).transpose(0, 1).reshape(shp)
    return w


def _native_qkv_to_neox(w: torch.Tensor, H: int, D: int) -> torch.Tensor:
    shp = w.shape
    return w.view(3, H, D, *shp[1:]).transpose(0, 1).reshape(shp)


def hf_to_native_plan(cfg: LMConfig, get, sd_keys=()) -> dict:
    """native name -> zero-arg producer of that tensor. ``get(k)`` reads HF key
    ``k`` (prefix-free). Lazy so tensor-parallel loading can materialise one
    tensor at a time and keep only its shard (BLOOM-176B does not fit in host
    memory per rank)."""
    H, D = cfg.n_heads, cfg.head_dim
    a = cfg.arch
    plan = {}

    def put(nk, fn):
        plan[nk] = fn

    def direct(nk, hk):
        plan[nk] = lambda hk=hk: get(hk)

    def cat3(nk, fmt):
        plan[nk] = lambda fmt=fmt: torch.cat([get(fmt.format(n)) for n in ("q", "k", "v")], 0)

    def tr(nk, hk):
        plan[nk] = lambda hk=hk: get(hk).t().contiguous()

    def neox(nk, hk):
        plan[nk] = lambda hk=hk: _neox_qkv_to_native(get(hk), H, D)

    if a in ("gptj", "gpt2", "gpt_neo"):
        direct("wte.weight", "wte.weight")
        if cfg.learned_pos:
            direct("wpe.weight", "wpe.weight")
        for i in range(cfg.n_layers):
            p = f"h.{i}."
            for ln in ("ln_1",) + (() if cfg.shared_ln else ("ln_2",)):
                direct(p + ln + ".weight", p + ln + ".weight")
                direct(p + ln + ".bias", p + ln + ".bias")
            if a == "gptj":
                cat3(p + "attn.qkv.weight", p + "attn.{}_proj.weight")
                direct(p + "attn.out.weight", p + "attn.out_proj.weight")
                for n in ("fc_in", "fc_out"):
                    direct(p + f"mlp.{n}.weight", p + f"mlp.{n}.weight")
                    direct(p + f"mlp.{n}.bias", p + f"mlp.{n}.bias")
            elif a == "gpt2":
                tr(p + "attn.qkv.weight", p + "attn.c_attn.weight")
                direct(p + "attn.qkv.bias", p + "attn.c_attn.bias")
                tr(p + "attn.out.weight", p + "attn.c_proj.weight")
                direct(p + "attn.out.bias", p + "attn.c_proj.bias")
                tr(p + "mlp.fc_in.weight", p + "mlp.c_fc.weight")
                direct(p + "mlp.fc_in.bias", p + "mlp.c_fc.bias")
                tr(p + "mlp.fc_out.weight", p + "mlp.c_proj.weight")
                direct(p + "mlp.fc_out.bias", p + "mlp.c_proj.bias")
            else:  # gpt_neo
                cat3(p + "attn.qkv.weight", p + "attn.attention.{}_proj.weight")
                direct(p + "attn.out.weight", p + "attn.attention.out_proj.weight")
                direct(p + "attn.out.bias", p + "attn.attention.out_proj.bias")
                direct(p + "mlp.fc_in.weight", p + "mlp.c_fc.weight")
                direct(p + "mlp.fc_in.bias", p + "mlp.c_fc.bias")
                direct(p + "mlp.fc_out.weight", p + "mlp.c_proj.weight")
                direct(p + "mlp.fc_out.bias", p + "mlp.c_proj.bias")
        direct("ln_f.weight", "ln_f.weight")
        direct("ln_f.bias", "ln_f.bias")
        if not cfg.tie_embeddings:
            direct("lm_head.weight", "lm_head.weight")
            if cfg.lm_head_bias and "lm_head.bias" in sd_keys:
                direct("lm_head.bias", "lm_head.bias")
        return plan

    if a == "gpt_neox":
        direct("wte.weight", "embed_in.weight")
        for i in range(cfg.n_layers):
            s, p = f"layers.{i}.", f"h.{i}."
            for nn_, hn in (("ln_1", "input_layernorm"), ("ln_2", "post_attention_layernorm")):
                direct(p + nn_ + ".weight", s + hn + ".weight")
                direct(p + nn_ + ".bias", s + hn + ".bias")
            neox(p + "attn.qkv.weight", s + "attention.query_key_value.weight")
            neox(p + "attn.qkv.bias", s + "attention.query_key_value.bias")
            for nn_, hn in (("attn.out", "attention.dense"), ("mlp.fc_in", "mlp.dense_h_to_4h"),
                            ("mlp.fc_out", "mlp.dense_4h_to_h")):
                direct(p + nn_ + ".weight", s + hn + ".weight")
                direct(p + nn_ + ".bias", s + hn + ".bias")
        direct("ln_f.weight", "final_layer_norm.weight")
        direct("ln_f.bias", "final_layer_norm.bias")
        if not cfg.tie_embeddings:
            direct("lm_head.weight", "embed_out.weight" if "embed_out.weight" in sd_keys else "lm_head.weight")
        return plan

    if a == "xglm":
        direct("wte.weight", "embed_tokens.weight")
        for i in range(cfg.n_layers):
            s, p = f"layers.{i}.", f"h.{i}."
            for nn_, hn in (("ln_1", "self_attn_layer_norm"), ("ln_2", "final_layer_norm")):
                direct(p + nn_ + ".weight", s + hn + ".weight")
                direct(p + nn_ + ".bias", s + hn + ".bias")
            cat3(p + "attn.qkv.weight", s + "self_attn.{}_proj.weight")
            cat3(p + "attn.qkv.bias", s + "self_attn.{}_proj.bias")
            for nn_, hn in (("attn.out", "self_attn.out_proj"), ("mlp.fc_in", "fc1"), ("mlp.fc_out", "fc2")):
                direct(p + nn_ + ".weight", s + hn + ".weight")
                direct(p + nn_ + ".bias", s + hn + ".bias")
        direct("ln_f.weight", "layer_norm.weight")
        direct("ln_f.bias", "layer_norm.bias")
        if not cfg.tie_embeddings:
            direct("lm_head.weight", "lm_head.weight")
        return plan

    if a == "bloom":
        direct("wte.weight", "word_embeddings.weight")
        direct("emb_ln.weight", "word_embeddings_layernorm.weight")
        direct("emb_ln.bias", "word_embeddings_layernorm.bias")
        for i in range(cfg.n_layers):
            p = f"h.{i}."
            for nn_, hn in (("ln_1", "input_layernorm"), ("ln_2", "post_attention_layernorm")):
                direct(p + nn_ + ".weight", p + hn + ".weight")
                direct(p + nn_ + ".bias", p + hn + ".bias")
            neox(p + "attn.qkv.weight", p + "self_attention.query_key_value.weight")
            neox(p + "attn.qkv.bias", p + "self_attention.query_key_value.bias")
            for nn_, hn in (("attn.out", "self_attention.dense"), ("mlp.fc_in", "mlp.dense_h_to_4h"),
                            ("mlp.fc_out", "mlp.dense_4h_to_h")):
                direct(p + nn_ + ".weight", p + hn + ".weight")
                direct(p + nn_ + ".bias", p + hn + ".bias")
        direct("ln_f.weight", "ln_f.weight")
        direct("ln_f.bias", "ln_f.bias")
        return plan
    raise ValueError(a)


_PREFIXES = ("", "transformer.", "gpt_neox.", "model.")


def prefixed_getter(sd):
    """``get(k)`` over a mapping whose keys may carry an HF model prefix."""
    def get(k):
        for pre in _PREFIXES:
            if pre + k in sd:
                return sd[pre + k]
        raise KeyError(k)
    return get


def hf_to_native(sd: dict, cfg: LMConfig) -> dict:
    """Map an HF state dict onto CausalLM parameter names."""
    plan = hf_to_native_plan(cfg, prefixed_getter(sd), tuple(sd.keys()))
    return {k: f() for k, f in plan.items()}


def native_to_hf(sd: dict, cfg: LMConfig) -> dict:
    """Inverse of :func:`hf_to_native` (HF-loadable state dict)."""
    out = {}
    H, D, d = cfg.n_heads, cfg.head_dim, cfg.hidden
    a = cfg.arch
    if a in ("gptj", "gpt2", "gpt_neo"):
        out["transformer.wte.weight"] = sd["wte.weight"]
        if cfg.learned_pos:
            out["transformer.wpe.weight"] = sd["wpe.weight"]
        for i in range(cfg.n_layers):
            p, t = f"h.{i}.", f"transformer.h.{i}."
            out[t + "ln_1.weight"] = sd[p + "ln_1.weight"]
            out[t + "ln_1.bias"] = sd[p + "ln_1.bias"]
            if not cfg.shared_ln:
                out[t + "ln_2.weight"] = sd[p + "ln_2.weight"]
                out[t + "ln_2.bias"] = sd[p + "ln_2.bias"]
            qkv = sd[p + "attn.qkv.weight"]
            if a == "gptj":
                for n, w in zip(("q", "k", "v"), qkv.split(d, 0)):
                    out[t + f"attn.{n}_proj.weight"] = w.contiguous()
                out[t + "attn.out_proj.weight"] = sd[p + "attn.out.weight"]
                for n in ("fc_in", "fc_out"):
                    out[t + f"mlp.{n}.weight"] = sd[p + f"mlp.{n}.weight"]
                    out[t + f"mlp.{n}.bias"] = sd[p + f"mlp.{n}.bias"]
            elif a == "gpt2":
                out[t + "attn.c_attn.weight"] = qkv.t().contiguous()
                out[t + "attn.c_attn.bias"] = sd[p + "attn.qkv.bias"]
                out[t + "attn.c_proj.weight"] = sd[p + "attn.out.weight"].t().contiguous()
                out[t + "attn.c_proj.bias"] = sd[p + "attn.out.bias"]
                out[t + "mlp.c_fc.weight"] = sd[p + "mlp.fc_in.weight"].t().contiguous()
                out[t + "mlp.c_fc.bias"] = sd[p + "mlp.fc_in.bias"]
                out[t + "mlp.c_proj.weight"] = sd[p + "mlp.fc_out.weight"].t().contiguous()
                out[t + "mlp.c_proj.bias"] = sd[p + "mlp.fc_out.bias"]
            else:
                for n, w in zip(("q", "k", "v"), qkv.split(d, 0)):
                    out[t + f"attn.attention.{n}_proj.weight"] = w.contiguous()
                out[t + "attn.attention.out_proj.weight"] = sd[p + "attn.out.weight"]
                out[t + "attn.attention.out_proj.bias"] = sd[p + "attn.out.bias"]
                out[t + "mlp.c_fc.weight"] = sd[p + "mlp.fc_in.weight"]
                out[t + "mlp.c_fc.bias"] = sd[p + "mlp.fc_in.bias"]
                out[t + "mlp.c_proj.weight"] = sd[p + "mlp.fc_out.weight"]
                out[t + "mlp.c_proj.bias"] = sd[p + "mlp.fc_out.bias"]
        out["transformer.ln_f.weight"] = sd["ln_f.weight"]
        out["transformer.ln_f.bias"] = sd["ln_f.bias"]
        if not cfg.tie_embeddings:
            out["lm_head.weight"] = sd["lm_head.weight"]
            if "lm_head.bias" in sd:
                out["lm_head.bias"] = sd["lm_head.bias"]
        return out
    if a == "gpt_neox":
        out["gpt_neox.embed_in.weight"] = sd["wte.weight"]
        for i in range(cfg.n_layers):
            p, t = f"h.{i}.", f"gpt_neox.layers.{i}."
            out[t + "input_layernorm.weight"] = sd[p + "ln_1.weight"]
            out[t + "input_layernorm.bias"] = sd[p + "ln_1.bias"]
            out[t + "post_attention_layernorm.weight"] = sd[p + "ln_2.weight"]
            out[t + "post_attention_layernorm.bias"] = sd[p + "ln_2.bias"]
            out[t + "attention.query_key_value.weight"] = _native_qkv_to_neox(sd[p + "attn.qkv.weight"], H, D)
            out[t + "attention.query_key_value.bias"] = _native_qkv_to_neox(sd[p + "attn.qkv.bias"], H, D)
            out[t + "attention.dense.weight"] = sd[p + "attn.out.weight"]
            out[t + "attention.dense.bias"] = sd[p + "attn.out.bias"]
            out[t + "mlp.dense_h_to_4h.weight"] = sd[p + "mlp.fc_in.weight"]
            out[t + "mlp.dense_h_to_4h.bias"] = sd[p + "mlp.fc_in.bias"]
            out[t + "mlp.dense_4h_to_h.weight"] = sd[p + "mlp.fc_out.weight"]
            out[t + "mlp.dense_4h_to_h.bias"] = sd[p + "mlp.fc_out.bias"]
        out["gpt_neox.final_layer_norm.weight"] = sd["ln_f.weight"]
        out["gpt_neox.final_layer_norm.bias"] = sd["ln_f.bias"]
        if not cfg.tie_embeddings:
            out["embed_out.weight"] = sd["lm_head.weight"]
        return out
    if a == "xglm":
        out["model.embed_tokens.weight"] = sd["wte.weight"]
        for i in range(cfg.n_layers):
            p, t = f"h.{i}.", f"model.layers.{i}."
            out[t + "self_attn_layer_norm.weight"] = sd[p + "ln_1.weight"]
            out[t + "self_attn_layer_norm.bias"] = sd[p + "ln_1.bias"]
            out[t + "final_layer_norm.weight"] = sd[p + "ln_2.weight"]
            out[t + "final_layer_norm.bias"] = sd[p + "ln_2.bias"]
            for n, w, b in zip(("q", "k", "v"), sd[p + "attn.qkv.weight"].split(d, 0), sd[p + "attn.qkv.bias"].split(d, 0)):
                out[t + f"self_attn.{n}_proj.weight"] = w.contiguous()
                out[t + f"self_attn.{n}_proj.bias"] = b.contiguous()
            for nn_, hn in (("attn.out", "self_attn.out_proj"), ("mlp.fc_in", "fc1"), ("mlp.fc_out", "fc2")):
                out[t + hn + ".weight"] = sd[p + nn_ + ".weight"]
                out[t + hn + ".bias"] = sd[p + nn_ + ".bias"]
        out["model.layer_norm.weight"] = sd["ln_f.weight"]
        out["model.layer_norm.bias"] = sd["ln_f.bias"]
        if not cfg.tie_embeddings:
            out["lm_head.weight"] = sd["lm_head.weight"]
        return out
    if a == "bloom":
        out["transformer.word_embeddings.weight"] = sd["wte.weight"]
        out["transformer.word_embeddings_layernorm.weight"] = sd["emb_ln.weight"]
        out["transformer.word_embeddings_layernorm.bias"] = sd["emb_ln.bias"]
        for i in range(cfg.n_layers):
            p, t = f"h.{i}.", f"transformer.h.{i}."
            out[t + "input_layernorm.weight"] = sd[p + "ln_1.weight"]
            out[t + "input_layernorm.bias"] = sd[p + "ln_1.bias"]
            out[t + "post_attention_layernorm.weight"] = sd[p + "ln_2.weight"]
            out[t + "post_attention_layernorm.bias"] = sd[p + "ln_2.bias"]
            out[t + "self_attention.query_key_value.weight"] = _native_qkv_to_neox(sd[p + "attn.qkv.weight"], H, D)
            out[t + "self_attention.query_key_value.bias"] = _native_qkv_to_neox(sd[p + "attn.qkv.bias"], H, D)
            out[t + "self_attention.dense.weight"] = sd[p + "attn.out.weight"]
            out[t + "self_attention.dense.bias"] = sd[p + "attn.out.bias"]
            out[t + "mlp.dense_h_to_4h.weight"] = sd[p + "mlp.fc_in.weight"]
            out[t + "mlp.dense_h_to_4h.bias"] = sd[p + "mlp.fc_in.bias"]
            out[t + "mlp.dense_4h_to_h.weight"] = sd[p + "mlp.fc_out.weight"]
            out[t + "mlp.dense_4h_to_h.bias"] = sd[p + "mlp.fc_out.bias"]
        out["transformer.ln_f.weight"] = sd["ln_f.weight"]
        out["transformer.ln_f.bias"] = sd["ln_f.bias"]
        return out
    raise ValueError(a)


_IGNORED = re.compile(r"(\.attn\.bias|\.attn\.masked_bias|rotary_emb\.inv_freq|\.attention\.bias|"
                      r"\.attention\.masked_bias|embed_positions\.weights)$")


def is_ignorable_hf_key(k: str) -> bool:
    return bool(_IGNORED.search(k))
