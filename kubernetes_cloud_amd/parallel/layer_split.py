"""Layer-split ("device_map") model placement -- the fallback the reference's
BLOOM-176B accelerate predictor uses (online-inference/bloom-176b/model/bloom.py:11,46:
``from_pretrained(..., device_map="auto", max_memory={0: '71GIB', ...})``).

Tensor parallelism (``parallel.tensor_parallel``) is the serving path on MI355X;
this is the fallback for when one process must hold a model bigger than one
GPU (or spill the tail of it to host memory): whole decoder blocks are placed
on devices in order under per-device byte budgets, each block's weights stream
straight from the safetensors files onto its device (no full host copy), and
forward pre-hooks move the hidden state across device boundaries. The serving
engine (``engine.runner.ModelRunner``) detects the split and keeps every
layer's KV cache on that layer's device.

Placement groups: ``embed`` (wte / wpe / emb_ln) first, then ``h.0`` ...,
then ``head`` (ln_f / lm_head). A tied LM head reads ``wte.weight``, so the
head group then sits with the embedding and the hidden state returns to the
first device for the logits.
"""
from __future__ import annotations

import re

import torch

_UNITS = {"": 1, "B": 1, "KB": 10**3, "MB": 10**6, "GB": 10**9, "TB": 10**12,
          "KIB": 2**10, "MIB": 2**20, "GIB": 2**30, "TIB": 2**40}


def parse_size(v) -> int:
    """``71GIB`` / ``'500MB'`` / ``1024`` -> bytes (accelerate's max_memory syntax)."""
    if isinstance(v, (int, float)):
        return int(v)
    m = re.fullmatch(r"\s*([0-9.]+)\s*([A-Za-z]*)\s*", str(v))
    if not m or m.group(2).upper() not in _UNITS:
        raise ValueError(f"bad size {v!r}")
    return int(float(m.group(1)) * _UNITS[m.group(2).upper()])


def _dev(k) -> torch.device:
    if isinstance(k, int) or (isinstance(k, str) and k.isdigit()):
        return torch.device("cuda", int(k))
    return torch.device(k)


def parse_max_memory(spec) -> dict:
    """``{0: '71GIB', 'cpu': '200GIB'}`` or ``"0:71GIB,1:71GIB,cpu:200GIB"`` -> {device: bytes}."""
    if isinstance(spec, str):
        spec = dict(item.split(":", 1) for item in spec.split(",") if item.strip())
    return {_dev(k): parse_size(v) for k, v in spec.items()}


def _groups(model) -> list[tuple[str, list[str]]]:
    g = [("embed", [n for n in ("wte", "wpe", "emb_ln") if getattr(model, n, None) is not None])]
    g += [(f"h.{i}", [f"h.{i}"]) for i in range(len(model.h))]
    g.append(("head", [n for n in ("ln_f", "lm_head") if getattr(model, n, None) is not None]))
    return g


def _nbytes(mod, dtype) -> int:
    es = torch.empty(0, dtype=dtype).element_size()
    return sum(p.numel() * es for p in mod.parameters())


def plan_device_map(model, max_memory, dtype: torch.dtype = torch.bfloat16) -> dict:
    """Greedy in-order placement of the placement groups under ``max_memory``
    (devices in the given order). -> {module name: torch.device}."""
    budget = parse_max_memory(max_memory)
    devs = list(budget)
    if not devs:
        raise ValueError("empty max_memory")
    used = {d: 0 for d in devs}
    tied = getattr(model, "lm_head", None) is None
    out, cur = {}, 0
    for gname, names in _groups(model):
        size = sum(_nbytes(model.get_submodule(n), dtype) for n in names)
        if gname == "head" and tied:
            d = out["wte"]  # the tied head needs wte.weight
            used[d] += size
        else:
            while used[devs[cur]] + size > budget[devs[cur]] and cur + 1 < len(devs):
                cur += 1
            d = devs[cur]
            if used[d] + size > budget[d]:
                raise MemoryError(f"{gname} ({size} B) does not fit in max_memory {max_memory}")
            used[d] += size
        for n in names:
            out[n] = d
    return out


def _move(x, dev):
    if isinstance(x, torch.Tensor):
        return x.to(dev, non_blocking=True) if x.device != dev else x
    if isinstance(x, tuple):
        return tuple(_move(v, dev) for v in x)
    if isinstance(x, list):
        return [_move(v, dev) for v in x]
    if isinstance(x, dict):
        return {k: _move(v, dev) for k, v in x.items()}
    return x


def _align_hook(dev):
    def hook(mod, args, kwargs):
        return _move(args, dev), _move(kwargs, dev)
    return hook


def dispatch_model(model, device_map: dict):
    """Move each mapped module to its device and make it pull its inputs there."""
    from ..models.causal_lm import alibi_slopes
    for name, dev in device_map.items():
        mod = model.get_submodule(name)
        mod.to(dev)
        mod.register_forward_pre_hook(_align_hook(dev), with_kwargs=True)
    if model.cfg.alibi:
        for i, blk in enumerate(model.h):
            blk.attn.alibi = alibi_slopes(model.cfg.n_heads).to(device_map[f"h.{i}"])
    model.hf_device_map = {k: str(v) for k, v in device_map.items()}
    return model


@torch.no_grad()
def load_layer_split(path: str, max_memory, dtype: torch.dtype = torch.bfloat16, device_map: dict | None = None):
    """Build the HF checkpoint at ``path`` split over devices; every tensor is
    read lazily from the safetensors files straight onto its device."""
    from ..models.causal_lm import CausalLM
    from ..models.config import LMConfig
    from ..models.hf_convert import hf_to_native_plan, prefixed_getter
    from .tensor_parallel import _LazySafetensors
    cfg = LMConfig.from_pretrained(path)
    with torch.device("meta"):
        m = CausalLM(cfg)
    m = m.to(dtype)
    dmap = device_map or plan_device_map(m, max_memory, dtype)
    for name, dev in dmap.items():
        m.get_submodule(name).to_empty(device=dev)
    try:
        sd = _LazySafetensors(path)
        if not list(sd.keys()):
            raise FileNotFoundError
    except FileNotFoundError:
        from ..io.hf import read_hf_state_dict
        sd = read_hf_state_dict(path)
    params = dict(m.named_parameters())
    seen = set()
    for name, produce in hf_to_native_plan(cfg, prefixed_getter(sd), tuple(sd.keys())).items():
        if name in params:
            params[name].copy_(produce().to(dtype))
            seen.add(name)
    missing = [n for n in params if n not in seen]
    if missing:
        raise RuntimeError(f"layer-split load: missing {missing[:8]}")
    return dispatch_model(m.eval(), dmap)


__all__ = ["parse_size", "parse_max_memory", "plan_device_map", "dispatch_model", "load_layer_split"]
