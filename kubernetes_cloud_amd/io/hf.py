"""HF-compatible model directories: ``config.json`` + safetensors shards.

Reads what HF ``from_pretrained`` reads (safetensors, sharded safetensors with
``model.safetensors.index.json``, or ``pytorch_model*.bin`` loaded with
``weights_only=True``) and writes what it writes, so ``checkpoint-N/`` and
``final/`` (finetuner-workflow/finetuner/finetuner.py:1055-1062) stay loadable
by the reference's serving side.
"""
from __future__ import annotations

import glob
import json
import os

import torch

from ..models.causal_lm import CausalLM, build_model
from ..models.config import LMConfig
from ..models.hf_convert import hf_to_native, is_ignorable_hf_key, native_to_hf

SAFE_NAME = "model.safetensors"


def read_hf_state_dict(path: str, device="cpu") -> dict:
    from safetensors.torch import load_file

    idx = os.path.join(path, "model.safetensors.index.json")
    if os.path.exists(idx):
        with open(idx) as f:
            files = sorted(set(json.load(f)["weight_map"].values()))
        sd = {}
        for fn in files:
            sd.update(load_file(os.path.join(path, fn), device=str(device)))
        return sd
    st = os.path.join(path, SAFE_NAME)
    if os.path.exists(st):
        return load_file(st, device=str(device))
    bins = sorted(glob.glob(os.path.join(path, "pytorch_model*.bin")))
    if bins:
        sd = {}
        for b in bins:
            sd.update(torch.load(b, map_location=device, weights_only=True))
        return sd
    raise FileNotFoundError(f"no weights (safetensors / pytorch_model.bin) in {path}")


def has_weights(path: str) -> bool:
    return any(os.path.exists(os.path.join(path, n)) for n in
               (SAFE_NAME, "model.safetensors.index.json")) or bool(
        glob.glob(os.path.join(path, "pytorch_model*.bin")))


def load_pretrained(path: str, device="cpu", dtype=torch.bfloat16, random_init_if_missing=False,
                    cfg: LMConfig | None = None) -> CausalLM:
    cfg = cfg or LMConfig.from_pretrained(path)
    model = build_model(cfg, device=device, dtype=dtype, seed=0)
    if has_weights(path):
        sd = read_hf_state_dict(path)
        nat = hf_to_native(sd, cfg)
        missing, unexpected = model.load_state_dict({k: v.to(dtype) for k, v in nat.items()},
                                                    strict=False)
        missing = [m for m in missing if not m.endswith("alibi")]
        if missing:
            raise RuntimeError(f"missing weights in {path}: {missing[:8]}")
    elif not random_init_if_missing:
        raise FileNotFoundError(f"no weights in {path}")
    return model


def load_tensorized(uri: str, config_dir: str | None = None, device="cpu", dtype=torch.bfloat16,
                    threads: int = 8) -> tuple[CausalLM, dict]:
    """Build the model with no init and stream its weights from a ``.tensors``
    file or ``http(s)://`` / ``s3://`` URI straight into the (preallocated)
    parameters -- the reference's ``no_init_or_tensor`` + ``TensorDeserializer``
    path (finetuner.py:802-815, tensorizer-isvc load_model.py:46-59). The
    config comes from ``config_dir/config.json`` when present, else from the
    file's own metadata (written by ``serialize_causal_lm``). -> (model, stats)."""
    from ..models.causal_lm import alibi_slopes
    from .tensors import load_into_module, metadata
    if config_dir and os.path.exists(os.path.join(config_dir, "config.json")):
        cfg = LMConfig.from_pretrained(config_dir)
    else:
        meta = metadata(uri)
        if "config" not in meta:
            raise FileNotFoundError(f"{uri}: no config.json given and no config in the file metadata")
        cfg = LMConfig.from_hf(meta["config"])
    with torch.device("meta"):
        model = CausalLM(cfg)
    model = model.to(dtype).to_empty(device=device)  # cast on meta: no fp32 materialisation
    stats = load_into_module(model, uri, device=device, threads=threads)
    if cfg.alibi:
        for blk in model.h:
            blk.attn.alibi = alibi_slopes(cfg.n_heads).to(device)
    return model, stats


def serialize_causal_lm(model: CausalLM, path: str, dtype: torch.dtype | None = None) -> dict:
    """``.tensors`` of a causal LM with its HF config embedded (so a URI alone
    is enough to rebuild it), e.g. ``model.tensors`` / ``gptj.tensors``."""
    from .tensors import serialize
    hf_cfg = model.cfg.to_hf()
    hf_cfg["vocab_size"] = model.cfg.vocab_size
    sd = {k: v for k, v in model.state_dict().items() if not k.endswith("alibi")}
    return serialize(sd, path, dtype=dtype, metadata={"config": hf_cfg, "kind": "causal_lm"})


def save_pretrained(model: CausalLM, path: str, max_shard_bytes: int = 10 << 30):
    """Write config.json + (sharded) safetensors in HF naming."""
    from safetensors.torch import save_file

    os.makedirs(path, exist_ok=True)
    cfg = model.cfg
    hf_cfg = cfg.to_hf()
    hf_cfg["vocab_size"] = cfg.vocab_size
    hf_cfg.setdefault("torch_dtype", str(next(model.parameters()).dtype).replace("torch.", ""))
    with open(os.path.join(path, "config.json"), "w") as f:
        json.dump(hf_cfg, f, indent=2)
    sd = {k: v.detach() for k, v in model.state_dict().items() if not k.endswith("alibi")}
    hf = native_to_hf(sd, cfg)
    hf = {k: v.contiguous().cpu() for k, v in hf.items()}
    total = sum(v.numel() * v.element_size() for v in hf.values())
    if total <= max_shard_bytes:
        save_file(hf, os.path.join(path, SAFE_NAME), metadata={"format": "pt"})
        return
    shards, cur, cur_b = [], {}, 0
    for k, v in hf.items():
        b = v.numel() * v.element_size()
        if cur and cur_b + b > max_shard_bytes:
            shards.append(cur)
            cur, cur_b = {}, 0
        cur[k] = v
        cur_b += b
    if cur:
        shards.append(cur)
    wm = {}
    n = len(shards)
    for i, sh in enumerate(shards):
        fn = f"model-{i + 1:05d}-of-{n:05d}.safetensors"
        save_file(sh, os.path.join(path, fn), metadata={"format": "pt"})
        for k in sh:
            wm[k] = fn
    with open(os.path.join(path, "model.safetensors.index.json"), "w") as f:
        json.dump({"metadata": {"total_size": total}, "weight_map": wm}, f, indent=2)


def load_tokenizer(path: str, eot: str = "", pad: str = ""):
    """AutoTokenizer from the model dir with the reference's special-token
    defaults (finetuner.py:412-444): explicit --eot/--pad win, else the
    model's, else ``<|endoftext|>``."""
    from transformers import AutoTokenizer

    kw = {}
    if eot:
        kw["eos_token"] = eot
    if pad:
        kw["pad_token"] = pad
    tok = AutoTokenizer.from_pretrained(path, **kw)
    add = {}
    if tok.eos_token is None:
        add["eos_token"] = "<|endoftext|>"
    if tok.pad_token is None:
        add["pad_token"] = tok.eos_token or "<|endoftext|>"
    if add:
        tok.add_special_tokens(add)
    return tok


__all__ = ["read_hf_state_dict", "load_pretrained", "save_pretrained", "load_tokenizer", "load_tensorized",
           "serialize_causal_lm",
           "is_ignorable_hf_key"]
