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


def hf_to_native(sd: dict, cfg: LMConfig) -> dict:
    """Map an HF state dict onto CausalLM parameter names."""
    out = {}
    H, D = cfg.n_heads, cfg.head_dim
    a = cfg.arch
    # strip common prefixes
    def get(k):
        for pre in ("", "transformer.", "gpt_neox.", "model."):
            if pre + k in sd:
                return sd[pre + k]
        raise KeyError(k)

    def has(k):
        return any((pre + k) in sd for pre in ("", "transformer.", "gpt_neox.", "model."))

    if a in ("gptj", "gpt2", "gpt_neo"):
        out["wte.weight"] = get("wte.weight")
        if cfg.learned_pos:
            out["wpe.weight"] = get("wpe.weight")
        for i in range(cfg.n_layers):
            p = f"h.{i}."
            out[p + "ln_1.weight"] = get(p + "ln_1.weight")
            out[p + "ln_1.bias"] = get(p + "ln_1.bias")
            if not cfg.shared_ln:
                out[p + "ln_2.weight"] = get(p + "ln_2.weight")
                out[p + "ln_2.bias"] = get(p + "ln_2.bias")
            if a == "gptj":
                out[p + "attn.qkv.weight"] = torch.cat(
                    [get(p + f"attn.{n}_proj.weight") for n in ("q", "k", "v")], 0)
                out[p + "attn.out.weight"] = get(p + "attn.out_proj.weight")
                out[p + "mlp.fc_in.weight"] = get(p + "mlp.fc_in.weight")
                out[p + "mlp.fc_in.bias"] = get(p + "mlp.fc_in.bias")
                out[p + "mlp.fc_out.weight"] = get(p + "mlp.fc_out.weight")
                out[p + "mlp.fc_out.bias"] = get(p + "mlp.fc_out.bias")
            elif a == "gpt2":
                out[p + "attn.qkv.weight"] = get(p + "attn.c_attn.weight").t().contiguous()
                out[p + "attn.qkv.bias"] = get(p + "attn.c_attn.bias")
                out[p + "attn.out.weight"] = get(p + "attn.c_proj.weight").t().contiguous()
                out[p + "attn.out.bias"] = get(p + "attn.c_proj.bias")
                out[p + "mlp.fc_in.weight"] = get(p + "mlp.c_fc.weight").t().contiguous()
                out[p + "mlp.fc_in.bias"] = get(p + "mlp.c_fc.bias")
                out[p + "mlp.fc_out.weight"] = get(p + "mlp.c_proj.weight").t().contiguous()
                out[p + "mlp.fc_out.bias"] = get(p + "mlp.c_proj.bias")
            else:  # gpt_neo
                out[p + "attn.qkv.weight"] = torch.cat(
                    [get(p + f"attn.attention.{n}_proj.weight") for n in ("q", "k", "v")], 0)
                out[p + "attn.out.weight"] = get(p + "attn.attention.out_proj.weight")
                out[p + "attn.out.bias"] = get(p + "attn.attention.out_proj.bias")
                out[p + "mlp.fc_in.weight"] = get(p + "mlp.c_fc.weight")
                out[p + "mlp.fc_in.bias"] = get(p + "mlp.c_fc.bias")
                out[p + "mlp.fc_out.weight"] = get(p + "mlp.c_proj.weight")
                out[p + "mlp.fc_out.bias"] = get(p + "mlp.c_proj.bias")
        out["ln_f.weight"] = get("ln_f.weight")
        out["ln_f.bias"] = get("ln_f.bias")
        if not cfg.tie_embeddings:
            out["lm_head.weight"] = sd["lm_head.weight"]
            if cfg.lm_head_bias and "lm_head.bias" in sd:
                out["lm_head.bias"] = sd["lm_head.bias"]
        return out

    if a == "gpt_neox":
        out["wte.weight"] = get("embed_in.weight")
        for i in range(cfg.n_layers):
            s, p = f"layers.{i}.", f"h.{i}."
            out[p + "ln_1.weight"] = get(s + "input_layernorm.weight")
            out[p + "ln_1.bias"] = get(s + "input_layernorm.bias")
            out[p + "ln_2.weight"] = get(s + "post_attention_layernorm.weight")
            out[p + "ln_2.bias"] = get(s + "post_attention_layernorm.bias")
            out[p + "attn.qkv.weight"] = _neox_qkv_to_native(get(s + "attention.query_key_value.weight"), H, D)
            out[p + "attn.qkv.bias"] = _neox_qkv_to_native(get(s + "attention.query_key_value.bias"), H, D)
            out[p + "attn.out.weight"] = get(s + "attention.dense.weight")
            out[p + "attn.out.bias"] = get(s + "attention.dense.bias")
            out[p + "mlp.fc_in.weight"] = get(s + "mlp.dense_h_to_4h.weight")
            out[p + "mlp.fc_in.bias"] = get(s + "mlp.dense_h_to_4h.bias")
            out[p + "mlp.fc_out.weight"] = get(s + "mlp.dense_4h_to_h.weight")
            out[p + "mlp.fc_out.bias"] = get(s + "mlp.dense_4h_to_h.bias")
        out["ln_f.weight"] = get("final_layer_norm.weight")
        out["ln_f.bias"] = get("final_layer_norm.bias")
        if not cfg.tie_embeddings:
            out["lm_head.weight"] = sd["embed_out.weight"] if "embed_out.weight" in sd else sd["lm_head.weight"]
        return out

    if a == "bloom":
        out["wte.weight"] = get("word_embeddings.weight")
        out["emb_ln.weight"] = get("word_embeddings_layernorm.weight")
        out["emb_ln.bias"] = get("word_embeddings_layernorm.bias")
        for i in range(cfg.n_layers):
            p = f"h.{i}."
            out[p + "ln_1.weight"] = get(p + "input_layernorm.weight")
            out[p + "ln_1.bias"] = get(p + "input_layernorm.bias")
            out[p + "ln_2.weight"] = get(p + "post_attention_layernorm.weight")
            out[p + "ln_2.bias"] = get(p + "post_attention_layernorm.bias")
            out[p + "attn.qkv.weight"] = _neox_qkv_to_native(get(p + "self_attention.query_key_value.weight"), H, D)
            out[p + "attn.qkv.bias"] = _neox_qkv_to_native(get(p + "self_attention.query_key_value.bias"), H, D)
            out[p + "attn.out.weight"] = get(p + "self_attention.dense.weight")
            out[p + "attn.out.bias"] = get(p + "self_attention.dense.bias")
            out[p + "mlp.fc_in.weight"] = get(p + "mlp.dense_h_to_4h.weight")
            out[p + "mlp.fc_in.bias"] = get(p + "mlp.dense_h_to_4h.bias")
            out[p + "mlp.fc_out.weight"] = get(p + "mlp.dense_4h_to_h.weight")
            out[p + "mlp.fc_out.bias"] = get(p + "mlp.dense_4h_to_h.bias")
        out["ln_f.weight"] = get("ln_f.weight")
        out["ln_f.bias"] = get("ln_f.bias")
        return out
    raise ValueError(a)


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
                      r"\.attention\.masked_bias)$")


def is_ignorable_hf_key(k: str) -> bool:
    return bool(_IGNORED.search(k))
