"""KServe / Triton V2 inference protocol tensors (JSON + binary-data extension).

The FasterTransformer-on-Triton path of the reference
(online-inference/fastertransformer/client/example.py:126-152) talks to the
server with ``tritonclient``: its HTTP client sends tensors with the binary
extension (JSON header whose length is in ``Inference-Header-Content-Length``,
followed by raw little-endian tensor bytes) and, when no outputs are named,
asks for binary outputs (``binary_data_output``). This module decodes and
encodes both forms so that client works unchanged against our server.
"""
from __future__ import annotations

import json
import struct

import numpy as np

HEADER = "inference-header-content-length"

_DT = {
    "BOOL": np.bool_, "UINT8": np.uint8, "UINT16": np.uint16, "UINT32": np.uint32, "UINT64": np.uint64,
    "INT8": np.int8, "INT16": np.int16, "INT32": np.int32, "INT64": np.int64, "FP16": np.float16,
    "FP32": np.float32, "FP64": np.float64, "BYTES": np.object_,
}
_NP = {np.dtype(v).str if v is not np.object_ else "O": k for k, v in _DT.items()}


def triton_dtype(a: np.ndarray) -> str:
    if a.dtype == np.object_ or a.dtype.kind in ("S", "U"):
        return "BYTES"
    return _NP[np.dtype(a.dtype).str]


def _bytes_decode(raw: bytes) -> list:
    out, i = [], 0
    while i < len(raw):
        (n,) = struct.unpack_from("<I", raw, i)
        out.append(raw[i + 4:i + 4 + n])
        i += 4 + n
    return out


def _bytes_encode(a: np.ndarray) -> bytes:
    parts = []
    for x in a.reshape(-1):
        b = x if isinstance(x, bytes) else str(x).encode()
        parts.append(struct.pack("<I", len(b)) + b)
    return b"".join(parts)


def decode_request(body: bytes, header_len: int | None) -> tuple[dict, dict]:
    """-> (request json, {input name: ndarray})."""
    if header_len is None:
        req = json.loads(body or b"{}")
        tail = b""
    else:
        req = json.loads(body[:header_len])
        tail = body[header_len:]
    tensors, off = {}, 0
    for inp in req.get("inputs", []):
        name, shape, dt = inp["name"], [int(s) for s in inp["shape"]], inp["datatype"]
        params = inp.get("parameters") or {}
        if "binary_data_size" in params:
            n = int(params["binary_data_size"])
            raw = tail[off:off + n]
            off += n
            if dt == "BYTES":
                arr = np.array(_bytes_decode(raw), dtype=np.object_).reshape(shape)
            else:
                arr = np.frombuffer(raw, dtype=_DT[dt]).reshape(shape).copy()
        else:
            data = inp.get("data", [])
            if dt == "BYTES":
                arr = np.array([d.encode() if isinstance(d, str) else d for d in np.ravel(data)],
                               dtype=np.object_).reshape(shape)
            else:
                arr = np.array(data, dtype=_DT[dt]).reshape(shape)
        tensors[name] = arr
    return req, tensors


def encode_response(model_name: str, outputs: dict, req: dict, model_version: str = "1",
                    request_id: str | None = None) -> tuple[bytes, dict]:
    """-> (body, extra headers). Binary encoding when the request asked for it
    (per output ``binary_data`` or request-level ``binary_data_output``)."""
    want = {o["name"]: o for o in req.get("outputs", []) or []}
    all_binary = bool((req.get("parameters") or {}).get("binary_data_output", False))
    names = list(want) if want else list(outputs)
    js, blobs = [], []
    for name in names:
        a = np.asarray(outputs[name])
        ent = {"name": name, "datatype": triton_dtype(a), "shape": list(a.shape)}
        binary = all_binary
        if name in want:
            binary = bool((want[name].get("parameters") or {}).get("binary_data", all_binary))
        if binary:
            raw = _bytes_encode(a) if ent["datatype"] == "BYTES" else np.ascontiguousarray(a).tobytes()
            ent["parameters"] = {"binary_data_size": len(raw)}
            blobs.append(raw)
        else:
            if ent["datatype"] == "BYTES":
                ent["data"] = [x.decode() if isinstance(x, bytes) else str(x) for x in a.reshape(-1)]
            else:
                ent["data"] = a.reshape(-1).tolist()
        js.append(ent)
    resp = {"model_name": model_name, "model_version": model_version, "outputs": js}
    if request_id or req.get("id"):
        resp["id"] = request_id or req.get("id")
    head = json.dumps(resp).encode()
    if blobs:
        return head + b"".join(blobs), {"Inference-Header-Content-Length": str(len(head))}
    return head, {}


def encode_request(inputs: dict, outputs: list | None = None, binary: bool = True,
                   binary_output: bool = True) -> tuple[bytes, dict]:
    """Client side (tests / load generator): the tritonclient wire format."""
    js, blobs = [], []
    for name, a in inputs.items():
        a = np.asarray(a)
        ent = {"name": name, "shape": list(a.shape), "datatype": triton_dtype(a)}
        if binary:
            raw = _bytes_encode(a) if ent["datatype"] == "BYTES" else np.ascontiguousarray(a).tobytes()
            ent["parameters"] = {"binary_data_size": len(raw)}
            blobs.append(raw)
        else:
            ent["data"] = a.reshape(-1).tolist()
        js.append(ent)
    req = {"inputs": js}
    if outputs:
        req["outputs"] = [{"name": n, "parameters": {"binary_data": binary_output}} for n in outputs]
    else:
        req["parameters"] = {"binary_data_output": binary_output}
    head = json.dumps(req).encode()
    hdr = {"Inference-Header-Content-Length": str(len(head))} if blobs else {}
    return head + b"".join(blobs), hdr


def decode_response(body: bytes, header_len: int | None) -> dict:
    """Client side: -> {output name: ndarray}."""
    head =json.loads(body[:header_len] if header_len else body)
    tail = body[header_len:] if header_len else b""
    out, off = {}, 0
    for o in head.get("outputs", []):
        params = o.get("parameters") or {}
        shape, dt = o["shape"], o["datatype"]
        if "binary_data_size" in params:
            n = int(params["binary_data_size"])
            raw = tail[off:off + n]
            off += n
            out[o["name"]] = (np.array(_bytes_decode(raw), dtype=np.object_).reshape(shape) if dt == "BYTES"
                              else np.frombuffer(raw, dtype=_DT[dt]).reshape(shape))
        else:
            out[o["name"]] = np.array(o["data"], dtype=_DT[dt] if dt != "BYTES" else np.object_).reshape(shape)
    return out


__all__ = ["decode_request", "encode_response", "encode_request", "decode_response", "triton_dtype", "HEADER"]
