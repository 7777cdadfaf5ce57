"""Flax ``msgpack`` checkpoints (``flax_model.msgpack``) without JAX.

The reference's DALL·E mini service loads ``DalleBart.from_pretrained`` and
``VQModel.from_pretrained`` Flax checkpoints (online-inference/dalle-mini/
model/service.py:71,84), written by ``flax.serialization.msgpack_serialize``:
a msgpack map tree whose leaves are ExtType records

* code 1 (ndarray): ``msgpack.packb((shape, dtype_name, C-order bytes))``,
* code 2 (native complex): ``msgpack.packb((real, imag))``,
* code 3 (numpy scalar): as code 1 with shape ``()``,

and arrays past ~1 GiB split as ``{"__msgpack_chunked_array__": True,
"shape": ..., "chunks": {"0": ..., "1": ...}}`` maps. ``read`` returns the same
tree with torch tensors (bfloat16 included, which numpy lacks); ``write`` emits
the identical encoding (tests, conversions). Pure data: decoding runs nothing
from the file.
"""
from __future__ import annotations

import math

import msgpack
import numpy as np
import torch

_NDARRAY, _COMPLEX, _SCALAR = 1, 2, 3
_CHUNKED = "__msgpack_chunked_array__"
MAX_CHUNK = 2 ** 30 - 2 ** 10  # flax.serialization._MAX_CHUNK_SIZE

_TORCH = {"float32": torch.float32, "float16": torch.float16, "bfloat16": torch.bfloat16,
          "float64": torch.float64, "int32": torch.int32, "int64": torch.int64, "int8": torch.int8,
          "uint8": torch.uint8, "int16": torch.int16, "bool": torch.bool}


def _shape_of(shape) -> tuple:
    """A chunked array's shape: flax writes a tuple as {"0": d0, "1": d1, ...}; a list is accepted too."""
    if isinstance(shape, dict):
        return tuple(int(shape[str(i)]) for i in range(len(shape)))
    return tuple(int(d) for d in shape)


def _array_from_bytes(data: bytes) -> torch.Tensor:
    shape, name, buf = msgpack.unpackb(data, raw=True)
    name = name.decode() if isinstance(name, bytes) else name
    dt = _TORCH.get(name)
    if dt is None:
        raise ValueError(f"unsupported dtype {name!r} in msgpack checkpoint")
    n = math.prod(shape)
    if n == 0:
        return torch.empty(tuple(shape), dtype=dt)
    t = torch.frombuffer(bytearray(buf), dtype=dt, count=n)
    return t.reshape(tuple(shape))


def _ext_hook(code: int, data: bytes):
    if code in (_NDARRAY, _SCALAR):
        return _array_from_bytes(data)
    if code == _COMPLEX:
        re, im = msgpack.unpackb(data)
        return complex(re, im)
    return msgpack.ExtType(code, data)


def _unchunk(tree):
    if isinstance(tree, dict):
        if tree.get(_CHUNKED):
            chunks = [tree["chunks"][str(i)] for i in range(len(tree["chunks"]))]
            return torch.cat([c.reshape(-1) for c in chunks]).reshape(_shape_of(tree["shape"]))
        return {k: _unchunk(v) for k, v in tree.items()}
    return tree


def loads(data: bytes) -> dict:
    return _unchunk(msgpack.unpackb(data, ext_hook=_ext_hook, raw=False, strict_map_key=False))


def read(path: str) -> dict:
    with open(path, "rb") as f:
        return loads(f.read())


def _array_bytes(t) -> bytes:
    if isinstance(t, torch.Tensor):
        t = t.detach().cpu().contiguous()
        name = str(t.dtype).replace("torch.", "")
        raw = t.view(torch.uint8).numpy().tobytes() if t.numel() else b""
        return msgpack.packb((list(t.shape), name, raw), use_bin_type=True)
    a = np.ascontiguousarray(t)
    return msgpack.packb((list(a.shape), a.dtype.name, a.tobytes("C")), use_bin_type=True)


def _default(x):
    if isinstance(x, (torch.Tensor, np.ndarray)):
        return msgpack.ExtType(_NDARRAY, _array_bytes(x))
    if isinstance(x, np.generic):
        return msgpack.ExtType(_SCALAR, _array_bytes(np.asarray(x)))
    if isinstance(x, complex):
        return msgpack.ExtType(_COMPLEX, msgpack.packb((x.real, x.imag)))
    raise TypeError(f"cannot serialise {type(x).__name__}")


def _chunk(tree, max_chunk: int):
    if isinstance(tree, dict):
        return {k: _chunk(v, max_chunk) for k, v in tree.items()}
    if isinstance(tree, torch.Tensor) and tree.numel() * tree.element_size() > max_chunk:
        flat = tree.reshape(-1)
        per = max(1, max_chunk // tree.element_size())
        parts = {str(i): flat[o:o + per].clone() for i, o in enumerate(range(0, flat.numel(), per))}
        # flax stores the shape tuple through its tuple -> {"0": d0, "1": d1, ...} state-dict mapping
        return {_CHUNKED: True, "shape": {str(i): int(d) for i, d in enumerate(tree.shape)}, "chunks": parts}
    return tree


def dumps(tree: dict, max_chunk: int = MAX_CHUNK) -> bytes:
    return msgpack.packb(_chunk(tree, max_chunk), default=_default, use_bin_type=True)


def write(tree: dict, path: str, max_chunk: int = MAX_CHUNK) -> None:
    with open(path, "wb") as f:
        f.write(dumps(tree, max_chunk))


def flatten(tree: dict, prefix: str = "") -> dict:
    """{"a": {"b": t}} -> {"a/b": t}."""
    out = {}
    for k, v in tree.items():
        key = f"{prefix}/{k}" if prefix else str(k)
        if isinstance(v, dict):
            out.update(flatten(v, key))
        else:
            out[key] = v
    return out


def unflatten(flat: dict) -> dict:
    tree: dict = {}
    for key, v in flat.items():
        node = tree
        parts = key.split("/")
        for p in parts[:-1]:
            node = node.setdefault(p, {})
        node[parts[-1]] = v
    return tree


__all__ = ["read", "write", "loads", "dumps", "flatten", "unflatten"]
