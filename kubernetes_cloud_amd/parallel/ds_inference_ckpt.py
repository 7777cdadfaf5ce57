"""Pre-sharded DeepSpeed-Inference TP checkpoints (S5 / N7).

The reference's BLOOM-176B DeepSpeed deployment serves
``microsoft/bloom-deepspeed-inference-fp16`` (online-inference/
bloom-176b-deepspeed/files/isvc-patch.txt:85-92): an HF repo whose
``ds_inference_config.json`` lists ``checkpoints.non_tp`` (tensors every rank
holds whole) and ``checkpoints.tp`` (``tp_{rank}_{shard}.pt`` -- rank r's
slices of the tensor-parallel weights, ``tp_size`` ranks), in BLOOM's HF
parameter names. ``load_ds_inference_tp`` builds THIS framework's TP shard
(``parallel.tensor_parallel`` layout) from it for any world size that divides
or is a multiple of the checkpoint's ``tp_size``, reading one file at a time
(memory-mapped, ``weights_only``): a 176B checkpoint never sits in host memory.

Slice axes (Megatron column/row split, what TP inference engines store):
``query_key_value`` by heads (rows, HF [H, 3, D] interleave),
``dense_h_to_4h`` weight/bias by rows, ``self_attention.dense`` and
``dense_4h_to_h`` weights by columns; everything else is replicated.
``export_ds_inference`` writes the same layout from an HF directory (tests,
re-sharding). Rank r's files are found by position in ``checkpoints.tp``
(DeepSpeed's assignment, not the file names), and ``[tensor, dtype]`` list
values (how DeepSpeed's TP save stores ``query_key_value``) are unwrapped.
Parity with the published checkpoint itself is unpinned: it is not in the tree
and there is no network; the layout follows its config schema.
"""
from __future__ import annotations

import json
import os

import torch

from ..models.hf_convert import _PREFIXES, _native_qkv_to_neox, _neox_qkv_to_native

CONFIG = "ds_inference_config.json"


def is_ds_inference_dir(path: str) -> bool:
    return os.path.isfile(os.path.join(path, CONFIG))


def _hf_kind(hf_key: str) -> str | None:
    """TP slice kind of an HF BLOOM key: qkv / row (dim 0) / col (dim 1) / None."""
    if hf_key.endswith("self_attention.query_key_value.weight") or \
            hf_key.endswith("self_attention.query_key_value.bias"):
        return "qkv"
    if hf_key.endswith("mlp.dense_h_to_4h.weight") or hf_key.endswith("mlp.dense_h_to_4h.bias"):
        return "row"
    if hf_key.endswith("self_attention.dense.weight") or hf_key.endswith("mlp.dense_4h_to_h.weight"):
        return "col"
    return None


def _strip(k: str) -> str:
    for p in _PREFIXES:
        if p and k.startswith(p):
            return k[len(p):]
    return k


def export_ds_inference(model_or_dir, out_dir: str, tp_size: int, shards_per_rank: int = 1,
                        dtype: torch.dtype = torch.float16) -> str:
    """Write an HF BLOOM model as a DeepSpeed-Inference TP checkpoint."""
    from ..io.hf import load_pretrained
    from ..models.hf_convert import native_to_hf
    m = load_pretrained(model_or_dir, dtype=dtype) if isinstance(model_or_dir, str) else model_or_dir
    cfg = m.cfg
    H, D = cfg.n_heads, cfg.head_dim
    hf = native_to_hf({k: v for k, v in m.state_dict().items() if not k.endswith("alibi")}, cfg)
    os.makedirs(out_dir, exist_ok=True)
    non_tp, tp = {}, [dict() for _ in range(tp_size)]
    for k, v in hf.items():
        kind = _hf_kind(k)
        v = v.to(dtype)
        if kind is None:
            non_tp[k] = v.contiguous()
        elif kind == "qkv":
            nat = _neox_qkv_to_native(v, H, D).view(3, H, D, *v.shape[1:])
            Hl = H // tp_size
            for r in range(tp_size):
                s = nat[:, r * Hl:(r + 1) * Hl].reshape(3 * Hl * D, *v.shape[1:])
                tp[r][k] = _native_qkv_to_neox(s, Hl, D).contiguous()
        else:
            dim = 0 if kind == "row" else 1
            for r, s in enumerate(v.chunk(tp_size, dim=dim)):
                tp[r][k] = s.contiguous()
    torch.save(non_tp, os.path.join(out_dir, "non-tp.pt"))
    names = []
    for s in range(shards_per_rank):  # partition-major, as DeepSpeed's TP save lists them
        for r in range(tp_size):
            keys = sorted(tp[r])
            part = {k: tp[r][k] for k in keys[s::shards_per_rank]}
            fn = f"tp_{r:02d}_{s:02d}.pt"
            torch.save(part, os.path.join(out_dir, fn))
            names.append(fn)
    with open(os.path.join(out_dir, CONFIG), "w") as f:
        json.dump({"type": "BLOOM", "base_dir": ".", "checkpoints": {"non_tp": ["non-tp.pt"], "tp": names},
                   "version": 1.0, "parallelization": "tp", "tp_size": tp_size,
                   "dtype": str(dtype).replace("torch.", "")}, f, indent=1)
    with open(os.path.join(out_dir, "config.json"), "w") as f:
        json.dump(cfg.to_hf(), f, indent=1)
    return out_dir


def _tp_files_by_rank(files: list, tp_size: int) -> dict:
    """Checkpoint rank -> its files. DeepSpeed assigns ``checkpoints.tp`` by
    POSITION, partition-major: with n = len(files) / tp_size partitions, rank r
    reads files[i*tp_size + r] for i < n (its loader's ``ckpt_index = i *
    ckpt_mp_size + sd_offset``); file names carry no contract."""
    if not files:
        return {}
    if len(files) % tp_size:
        raise ValueError(f"{len(files)} tp checkpoint files do not split over tp_size {tp_size}")
    n = len(files) // tp_size
    return {r: [files[i * tp_size + r] for i in range(n)] for r in range(tp_size)}


def _unwrap(v):
    """DeepSpeed's TP save stores some entries (query_key_value) as
    ``[tensor, dtype]`` lists; take the tensor."""
    while isinstance(v, (list, tuple)):
        if not v:
            raise ValueError("empty list value in DS-inference checkpoint")
        v = v[0]
    if not isinstance(v, torch.Tensor):
        raise TypeError(f"unexpected checkpoint value {type(v).__name__}")
    return v


@torch.no_grad()
def load_ds_inference_tp(path: str, rank: int, world: int, group=None, device=None, dtype=torch.bfloat16):
    """This rank's TP shard (``tensor_parallel.tp_convert_`` layout) of a
    DeepSpeed-Inference checkpoint directory."""
    from ..models.causal_lm import CausalLM, alibi_slopes
    from ..models.config import LMConfig
    from ..models.hf_convert import hf_to_native_plan
    from .tensor_parallel import shard_native_tensor, tp_convert_
    with open(os.path.join(path, CONFIG)) as f:
        dsc = json.load(f)
    T = int(dsc.get("tp_size", 1))
    if not (T % world == 0 or world % T == 0):
        raise ValueError(f"world {world} incompatible with checkpoint tp_size {T}")
    cfg = LMConfig.from_pretrained(path)
    H, D = cfg.n_heads, cfg.head_dim
    base = os.path.join(path, dsc.get("base_dir", ".") or ".")
    ck = dsc["checkpoints"]

    def load(fn):
        return torch.load(os.path.join(base, fn), map_location="cpu", weights_only=True, mmap=True)

    # which checkpoint ranks feed this rank, and which sub-slice of them
    if T >= world:
        src_ranks, sub, nsub = list(range(rank * T // world, (rank + 1) * T // world)), 0, 1
    else:
        src_ranks, sub, nsub = [rank * T // world], rank % (world // T), world // T
    full: dict = {}
    for fn in ck.get("non_tp", []):
        full.update({_strip(k): _unwrap(v) for k, v in load(fn).items()})
    slices: dict = {}  # hf key -> {ckpt rank: tensor}
    by_rank = _tp_files_by_rank(list(ck.get("tp", [])), T)
    for r in src_ranks:
        for fn in by_rank.get(r, ()):
            for k, v in load(fn).items():
                slices.setdefault(_strip(k), {})[r] = _unwrap(v)

    Hs = H // T  # heads per checkpoint slice

    def tp_getter(hk):
        """Native-layout tensor covering this rank's part of HF key ``hk``
        (a concatenation of checkpoint slices, sub-sliced when world > T)."""
        parts = [slices[hk][r] for r in src_ranks]
        kind = _hf_kind(hk)
        if kind == "qkv":
            nat = [_neox_qkv_to_native(p, Hs, D).view(3, Hs, D, *p.shape[1:]) for p in parts]
            t = torch.cat(nat, 1)
            if nsub > 1:
                n = t.shape[1] // nsub
                t = t[:, sub * n:(sub + 1) * n]
            return t.reshape(-1, *parts[0].shape[1:])
        dim = 0 if kind == "row" else 1
        t = torch.cat(parts, dim)
        if nsub > 1:
            t = t.chunk(nsub, dim=dim)[sub]
        return t

    with torch.device("meta"):
        m = CausalLM(cfg)
    tp_convert_(m, rank, world, group)
    m = m.to(dtype).to_empty(device=device or "cpu")
    params = dict(m.named_parameters())

    def get_full(hk):
        if hk in full:
            return full[hk]
        raise KeyError(hk)

    plan = hf_to_native_plan(cfg, get_full, tuple(full) + tuple(slices))
    seen = set()
    for name, produce in plan.items():
        if name not in params:
            continue
        p = params[name]
        hk = _native_to_hf_key(name)
        if hk in slices:
            shard = tp_getter(hk)  # already this rank's part, native layout
        else:
            shard = shard_native_tensor(name, produce(), cfg, rank, world)
        if tuple(shard.shape) != tuple(p.shape):
            raise ValueError(f"{name}: shard {tuple(shard.shape)} != param {tuple(p.shape)}")
        p.copy_(shard.to(p.dtype))
        seen.add(name)
    if "lm_head.weight" in params and "lm_head.weight" not in seen:  # tied vocab-parallel head
        params["lm_head.weight"].copy_(shard_native_tensor("lm_head.weight", full["word_embeddings.weight"], cfg,
                                                           rank, world).to(dtype))
        seen.add("lm_head.weight")
    missing = [n for n in params if n not in seen]
    if missing:
        raise RuntimeError(f"DS-inference load: missing {missing[:8]}")
    if cfg.alibi:
        Hl = H // world
        for blk in m.h:
            blk.attn.alibi = alibi_slopes(H)[rank * Hl:(rank + 1) * Hl].to(m.wte.weight.device)
    return m


def _native_to_hf_key(name: str) -> str:
    """Native BLOOM param name -> HF key (prefix-free)."""
    mp = {"attn.qkv": "self_attention.query_key_value", "attn.out": "self_attention.dense",
          "mlp.fc_in": "mlp.dense_h_to_4h", "mlp.fc_out": "mlp.dense_4h_to_h", "ln_1": "input_layernorm",
          "ln_2": "post_attention_layernorm"}
    if name.startswith("h."):
        _, i, rest = name.split(".", 2)
        mod, _, leaf = rest.rpartition(".")
        return f"h.{i}.{mp.get(mod, mod)}.{leaf}"
    return {"wte.weight": "word_embeddings.weight", "emb_ln.weight": "word_embeddings_layernorm.weight",
            "emb_ln.bias": "word_embeddings_layernorm.bias"}.get(name, name)


__all__ = ["is_ds_inference_dir", "load_ds_inference_tp", "export_ds_inference"]
