"""``.tensors`` files: serializer + streaming deserializer (D3 / N17 / K25).

The reference serializes modules with tensorizer (stable-diffusion/serializer/
serialize.py:13-50 -> ``{encoder,vae,unet}.tensors``; tensorizer-isvc/
model-download/model_download.py:23-25 -> ``gptj.tensors``) and streams them
back with ``TensorDeserializer(plaid_mode=True)`` (load_model.py:56-59). The
tensorizer wire format is external and not in the tree, so this framework
defines its own layout behind the same file names:

    b"KCATNSR1" | u64 header_len | header JSON | pad to 4 KiB |
    tensor 0 data (4 KiB aligned) | tensor 1 data | ...

    header = {"format": "kca-tensors/1", "metadata": {...},
              "tensors": [{"name", "dtype", "shape", "offset", "nbytes"}, ...]}

Every tensor starts on a 4 KiB boundary so the native streamer can read it
with O_DIRECT into pinned buffers and ``hipMemcpyAsync`` it straight into the
preallocated HBM parameter (``csrc/io/tensor_stream.cpp``): no allocator work,
no module construction, no per-tensor Python on the hot path.
"""
from __future__ import annotations

import ctypes
import json
import os
import struct
import time

import numpy as np
import torch

MAGIC = b"KCATNSR1"
ALIGN = 4096
_DT = {
    torch.float32: "float32", torch.float16: "float16", torch.bfloat16: "bfloat16",
    torch.int64: "int64", torch.int32: "int32", torch.int16: "int16", torch.int8: "int8",
    torch.uint8: "uint8", torch.bool: "bool", torch.float64: "float64",
}
_TD = {v: k for k, v in _DT.items()}


def _align(x: int) -> int:
    return (x + ALIGN - 1) // ALIGN * ALIGN


def _flat_bytes(t: torch.Tensor) -> np.ndarray:
    t = t.detach().contiguous().cpu()
    if t.dtype == torch.bfloat16:
        t = t.view(torch.int16)
    elif t.dtype == torch.bool:
        t = t.view(torch.uint8)
    return t.numpy().reshape(-1).view(np.uint8)


def serialize(obj, path: str, dtype: torch.dtype | None = None, metadata: dict | None = None) -> dict:
    """Write a module / state dict. ``dtype`` casts floating tensors (e.g. fp16
    serving copies, like ``model_download.py``'s fp16 GPT-J)."""
    sd = obj.state_dict() if hasattr(obj, "state_dict") else dict(obj)
    entries, off = [], 0
    items = []
    for name, t in sd.items():
        if not isinstance(t, torch.Tensor):
            continue
        if dtype is not None and t.is_floating_point():
            t = t.to(dtype)
        nb = t.numel() * t.element_size()
        entries.append({"name": name, "dtype": _DT[t.dtype], "shape": list(t.shape), "offset": off,
                        "nbytes": nb})
        items.append(t)
        off = _align(off + nb)
    header = json.dumps({"format": "kca-tensors/1", "metadata": metadata or {}, "tensors": entries}).encode()
    data_start = _align(len(MAGIC) + 8 + len(header))
    tmp = path + ".tmp"
    with open(tmp, "wb") as f:
        f.write(MAGIC)
        f.write(struct.pack("<Q", len(header)))
        f.write(header)
        f.write(b"\0" * (data_start - f.tell()))
        for e, t in zip(entries, items):
            pos = data_start + e["offset"]
            if f.tell() < pos:
                f.write(b"\0" * (pos - f.tell()))
            f.write(_flat_bytes(t).tobytes())
        end = data_start + off
        if f.tell() < end:
            f.write(b"\0" * (end - f.tell()))
    os.replace(tmp, path)
    return {"bytes": off, "tensors": len(entries), "data_start": data_start}


def read_header(path: str) -> tuple[dict, int]:
    with open(path, "rb") as f:
        if f.read(8) != MAGIC:
            raise ValueError(f"{path}: not a kca .tensors file")
        (hl,) = struct.unpack("<Q", f.read(8))
        hdr = json.loads(f.read(hl))
    return hdr, _align(len(MAGIC) + 8 + hl)


def _stream(path: str, offs, lens, ptrs, device: torch.device, threads: int, chunk: int,
            odirect: bool, info: dict | None = None) -> tuple[float, float]:
    from . import native
    n = len(offs)
    a_off = (ctypes.c_longlong * n)(*offs)
    a_len = (ctypes.c_longlong * n)(*lens)
    a_ptr = (ctypes.c_void_p * n)(*ptrs)
    stats = (ctypes.c_double * 4)()
    lib = native.load()
    if device.type == "cuda":
        rc = lib.kca_stream_to_device(path.encode(), n, a_off, a_len, a_ptr,
                                      device.index if device.index is not None else torch.cuda.current_device(),
                                      threads, chunk, int(odirect), stats)
    else:
        rc = lib.kca_read_ranges(path.encode(), n, a_off, a_len, a_ptr, threads, chunk, stats)
    if rc != 0:
        raise IOError(f"native streamer failed on {path} (code {rc})")
    if info is not None and device.type == "cuda":  # which read path carried the payload
        info["odirect_bytes"], info["buffered_bytes"] = int(stats[2]), int(stats[3])
    return stats[0], stats[1]


def _python_read(path, offs, lens, tensors):
    t0 = time.perf_counter()
    with open(path, "rb") as f:
        for o, n, t in zip(offs, lens, tensors):
            f.seek(o)
            buf = f.read(n)
            src = torch.frombuffer(bytearray(buf), dtype=torch.uint8)
            t.view(-1).view(torch.uint8).copy_(src)
    return float(sum(lens)), time.perf_counter() - t0


def _header_any(path: str):
    from . import remote
    if remote.is_remote(path):
        return remote.read_header(path)
    hdr, start = read_header(path)
    return hdr, start, None


def load_into_module(module: torch.nn.Module, path: str, device=None, strict: bool = True,
                     threads: int = 8, chunk: int = 64 << 20, odirect: bool = True) -> dict:
    """Stream a ``.tensors`` file -- a local path, or an ``http(s)://`` /
    ``s3://`` URI (io/remote.py) -- into an existing module's parameters/buffers.

    Same-dtype tensors stream straight into the parameter storage; others go
    through a staging tensor and a cast. Returns {bytes, seconds, gbps}."""
    t_begin = time.perf_counter()
    hdr, data_start, rem = _header_any(path)
    own = dict(module.state_dict(keep_vars=True))
    dev = torch.device(device) if device is not None else next(module.parameters()).device
    offs, lens, ptrs, targets, casts = [], [], [], [], []
    seen = set()
    for e in hdr["tensors"]:
        name = e["name"]
        if name not in own:
            if strict:
                raise KeyError(f"{name} in {path} not in module")
            continue
        dst = own[name].data if isinstance(own[name], torch.nn.Parameter) else own[name]
        seen.add(name)
        if list(dst.shape) != e["shape"]:
            raise ValueError(f"{name}: shape {list(dst.shape)} != file {e['shape']}")
        src_dt = _TD[e["dtype"]]
        if dst.dtype == src_dt and dst.is_contiguous() and dst.device == dev:
            buf = dst
        else:
            buf = torch.empty(e["shape"], dtype=src_dt, device=dev)
            casts.append((buf, dst))
        if e["nbytes"]:
            offs.append(data_start + e["offset"])
            lens.append(e["nbytes"])
            ptrs.append(buf.data_ptr())
            targets.append(buf)
    if strict:
        missing = [k for k in own if k not in seen and not k.endswith("alibi")]
        if missing:
            raise KeyError(f"missing in {path}: {missing[:8]}")
    from . import native
    paths: dict = {}
    if rem is not None:
        from . import remote
        nbytes, secs = remote.stream(rem, offs, lens, ptrs, dev, threads=max(threads, 16),
                                     chunk=min(chunk, 16 << 20))
    elif native.available():
        nbytes, secs = _stream(path, offs, lens, ptrs, dev, threads, chunk, odirect, paths)
    else:
        if dev.type == "cuda":
            native.load()  # raises: never silently fall back on a GPU load
        nbytes, secs = _python_read(path, offs, lens, targets)
    with torch.no_grad():
        for buf, dst in casts:
            dst.copy_(buf)
    if dev.type == "cuda":
        torch.cuda.synchronize(dev)
    return {"bytes": nbytes, "seconds": secs, "gbps": nbytes / max(secs, 1e-9) / 1e9,
            "seconds_total": time.perf_counter() - t_begin, "source": "http" if rem is not None else "file", **paths}


def load_state_dict(path: str, device="cpu", threads: int = 8) -> dict:
    hdr, data_start, rem = _header_any(path)
    dev = torch.device(device)
    out, offs, lens, ptrs, ts = {}, [], [], [], []
    for e in hdr["tensors"]:
        t = torch.empty(e["shape"], dtype=_TD[e["dtype"]], device=dev)
        out[e["name"]] = t
        if e["nbytes"]:
            offs.append(data_start + e["offset"])
            lens.append(e["nbytes"])
            ptrs.append(t.data_ptr())
            ts.append(t)
    from . import native
    paths: dict = {}
    if rem is not None:
        from . import remote
        remote.stream(rem, offs, lens, ptrs, dev, threads=max(threads, 16))
    elif native.available():
        _stream(path, offs, lens, ptrs, dev, threads, 64 << 20, True)
    else:
        _python_read(path, offs, lens, ts)
    return out


def metadata(path: str) -> dict:
    return _header_any(path)[0].get("metadata", {})
