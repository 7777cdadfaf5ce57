"""Remote ``.tensors`` sources: ``http(s)://`` and ``s3://`` URIs (N17 / K25).

The reference streams weights straight from object storage with tensorizer's
``CURLStreamFile`` / ``open_stream`` (finetuner-workflow/finetuner/
finetuner.py:395-410 probes the public ``tensorized`` bucket and :802-815
loads from it; stable-diffusion/service/service.py:87-93;
tensorizer-isvc/tensorizer_hf_isvc/load_model.py:56-59). Here the transfer is
the native ranged-GET streamer (csrc/io/http_stream.cpp: N keep-alive
connections, pinned double buffers, hipMemcpyAsync into preallocated HBM);
this module resolves URIs, signs S3 requests and reads the file header.

* ``s3://bucket/key`` -> path-style ``{endpoint}/bucket/key``; endpoint from
  ``S3_ENDPOINT_URL`` / ``AWS_ENDPOINT_URL`` (default CoreWeave's accelerated
  endpoint, the one the reference probes); requests are anonymous unless
  ``AWS_ACCESS_KEY_ID`` / ``AWS_SECRET_ACCESS_KEY`` are set, then SigV4
  (``UNSIGNED-PAYLOAD``). S3 rejects header-signed requests older than 15
  minutes, so ``stream`` re-signs before every window of at most
  ``RESIGN_BYTES`` (2 GB: > 2 MB/s keeps a window inside the limit) and
  re-signs and retries once when a window comes back 403.
* TLS peers are verified against the system CA store (``KCA_TLS_VERIFY=0``
  disables it, e.g. for a self-signed test server).
"""
from __future__ import annotations

import ctypes
import datetime
import hashlib
import hmac
import json
import os
import struct
import urllib.parse
from dataclasses import dataclass

DEFAULT_S3_ENDPOINT = "https://accel-object.ord1.coreweave.com"
RESIGN_BYTES = 2 << 30
PUBLIC_TENSORIZED = "https://accel-object.ord1.coreweave.com/tensorized"


def is_remote(uri: str) -> bool:
    return isinstance(uri, str) and uri.split("://", 1)[0].lower() in ("http", "https", "s3")


@dataclass
class Remote:
    host: str
    port: int
    tls: bool
    path: str
    headers: str = ""
    verify: bool = True
    timeout_s: float = 30.0
    signer: object = None  # () -> fresh header block (SigV4), or None for anonymous / static headers

    def resign(self):
        if self.signer is not None:
            self.headers = self.signer()

    @property
    def url(self) -> str:
        scheme = "https" if self.tls else "http"
        return f"{scheme}://{self.host}:{self.port}{self.path}"


def _sigv4_headers(host: str, path: str, access: str, secret: str, region: str, token: str | None = None,
                   now: datetime.datetime | None = None) -> str:
    """AWS Signature V4 for a GET of ``path`` (query-less), payload unsigned."""
    now = now or datetime.datetime.now(datetime.timezone.utc)
    amz_date = now.strftime("%Y%m%dT%H%M%SZ")
    day = amz_date[:8]
    hdrs = {"host": host, "x-amz-content-sha256": "UNSIGNED-PAYLOAD", "x-amz-date": amz_date}
    if token:
        hdrs["x-amz-security-token"] = token
    names = sorted(hdrs)
    canon = "\n".join(["GET", urllib.parse.quote(path, safe="/~"), "",
                       "".join(f"{k}:{hdrs[k]}\n" for k in names), ";".join(names), "UNSIGNED-PAYLOAD"])
    scope = f"{day}/{region}/s3/aws4_request"
    to_sign = "\n".join(["AWS4-HMAC-SHA256", amz_date, scope, hashlib.sha256(canon.encode()).hexdigest()])

    def h(k, m):
        return hmac.new(k, m.encode(), hashlib.sha256).digest()
    key = h(h(h(h(("AWS4" + secret).encode(), day), region), "s3"), "aws4_request")
    sig = hmac.new(key, to_sign.encode(), hashlib.sha256).hexdigest()
    auth = (f"AWS4-HMAC-SHA256 Credential={access}/{scope}, SignedHeaders={';'.join(names)}, "
            f"Signature={sig}")
    out = {"x-amz-content-sha256": "UNSIGNED-PAYLOAD", "x-amz-date": amz_date, "Authorization": auth}
    if token:
        out["x-amz-security-token"] = token
    return "".join(f"{k}: {v}\r\n" for k, v in out.items())


def resolve(uri: str, timeout_s: float = 30.0) -> Remote:
    scheme, rest = uri.split("://", 1)
    scheme = scheme.lower()
    verify = os.environ.get("KCA_TLS_VERIFY", "1") not in ("0", "false", "no")
    if scheme == "s3":
        bucket, _, key = rest.partition("/")
        ep = os.environ.get("S3_ENDPOINT_URL") or os.environ.get("AWS_ENDPOINT_URL") or DEFAULT_S3_ENDPOINT
        if "://" not in ep:
            ep = "https://" + ep
        r = resolve(ep.rstrip("/") + "/" + bucket + "/" + key, timeout_s)
        access, secret = os.environ.get("AWS_ACCESS_KEY_ID"), os.environ.get("AWS_SECRET_ACCESS_KEY")
        if access and secret:
            region = os.environ.get("AWS_DEFAULT_REGION", os.environ.get("AWS_REGION", "us-east-1"))
            token = os.environ.get("AWS_SESSION_TOKEN")
            r.signer = lambda: _sigv4_headers(r.host, r.path, access, secret, region, token)
            r.resign()
        return r
    u = urllib.parse.urlsplit(uri)
    if scheme not in ("http", "https") or not u.hostname:
        raise ValueError(f"unsupported URI {uri!r} (http://, https://, s3://)")
    tls = scheme == "https"
    path = u.path or "/"
    if u.query:
        path += "?" + u.query
    return Remote(u.hostname, u.port or (443 if tls else 80), tls, path, "", verify, timeout_s)


def get_range(r: Remote, off: int, n: int) -> tuple[bytes, int]:
    """(bytes, total object size) of ``[off, off + n)``; raises IOError."""
    from . import native
    lib = native.load()
    buf = ctypes.create_string_buffer(n)
    total = ctypes.c_longlong(0)
    rc = lib.kca_http_get_range(r.host.encode(), r.port, int(r.tls), int(r.verify), r.path.encode(),
                                r.headers.encode(), off, n, buf, ctypes.byref(total), r.timeout_s)
    if rc != 0:
        raise IOError(f"GET {r.url} bytes={off}-{off + n - 1}: " + (f"HTTP {rc}" if rc >= 100 else f"error {rc}"))
    return buf.raw, total.value


def exists(uri: str, timeout_s: float = 5.0) -> bool:
    """One-byte ranged GET (the reference's ``CURLStreamFile(uri, end=1)`` probe
    and the workflow's ``curl -I`` check-model step)."""
    try:
        get_range(resolve(uri, timeout_s), 0, 1)
        return True
    except (IOError, OSError, ValueError):
        return False


def is_kca_object(uri: str, timeout_s: float = 5.0) -> bool:
    """True when the object at ``uri`` starts with this framework's ``.tensors`` magic (an
    8-byte ranged GET); False for a foreign object (e.g. a CoreWeave tensorizer file, whose
    wire format is not in the tree) or an unreachable one."""
    from .tensors import MAGIC
    try:
        head, _ = get_range(resolve(uri, timeout_s), 0, len(MAGIC))
    except (IOError, OSError, ValueError):
        return False
    return head[:len(MAGIC)] == MAGIC


def read_header(uri: str, timeout_s: float = 30.0) -> tuple[dict, int, Remote]:
    from .tensors import ALIGN, MAGIC
    r = resolve(uri, timeout_s)
    head, _ = get_range(r, 0, 16)
    if head[:8] != MAGIC:
        raise ValueError(f"{uri}: not a kca .tensors object")
    (hl,) = struct.unpack("<Q", head[8:16])
    body, _ = get_range(r, 16, hl)
    hdr = json.loads(body)
    return hdr, (16 + hl + ALIGN - 1) // ALIGN * ALIGN, r


def _windows(lens, limit: int):
    """Index ranges [i, j) of consecutive ranges summing to <= ``limit`` bytes
    (a single larger range gets a window of its own)."""
    i, acc = 0, 0
    for j, n in enumerate(lens):
        if j > i and acc + n > limit:
            yield i, j
            i, acc = j, 0
        acc += n
    if i < len(lens):
        yield i, len(lens)


def stream(r: Remote, offs, lens, ptrs, device, threads: int = 16, chunk: int = 16 << 20) -> tuple[float, float]:
    """Ranged GETs into device (``device.type == 'cuda'``) or host pointers.
    Signed sources are re-signed per window (and once more on a 403)."""
    if r.signer is None:
        return _stream(r, offs, lens, ptrs, device, threads, chunk)
    tot_b, tot_s = 0.0, 0.0
    for i, j in _windows(list(lens), RESIGN_BYTES):
        r.resign()
        try:
            b, s = _stream(r, offs[i:j], lens[i:j], ptrs[i:j], device, threads, chunk)
        except IOError as e:
            if "HTTP 403" not in str(e):
                raise
            r.resign()  # e.g. RequestTimeTooSkewed / expired signature: one fresh attempt
            b, s = _stream(r, offs[i:j], lens[i:j], ptrs[i:j], device, threads, chunk)
        tot_b, tot_s = tot_b + b, tot_s + s
    return tot_b, tot_s


def _stream(r: Remote, offs, lens, ptrs, device, threads: int = 16, chunk: int = 16 << 20) -> tuple[float, float]:
    import torch

    from . import native
    lib = native.load()
    n = len(offs)
    a_off = (ctypes.c_longlong * n)(*offs)
    a_len = (ctypes.c_longlong * n)(*lens)
    a_ptr = (ctypes.c_void_p * n)(*ptrs)
    stats = (ctypes.c_double * 2)()
    dev = -1
    if device.type == "cuda":
        dev = device.index if device.index is not None else torch.cuda.current_device()
    rc = lib.kca_http_stream(r.host.encode(), r.port, int(r.tls), int(r.verify), r.path.encode(),
                             r.headers.encode(), n, a_off, a_len, a_ptr, dev, threads, chunk, r.timeout_s, stats)
    if rc != 0:
        raise IOError(f"streaming {r.url} failed: " + (f"HTTP {rc}" if rc >= 100 else f"error {rc}"))
    return stats[0], stats[1]


def public_tensorized_uri(model: str, fp16: bool = False, timeout_s: float = 5.0) -> str | None:
    """The reference's public-bucket probe (finetuner.py:395-410): if
    ``{org}/{name}`` is published under the ``tensorized`` bucket, return its
    ``s3://`` URI (fp16 variant with ``fp16``), else None. ``KCA_TENSORIZED_BASE``
    overrides the probe base URL; ``KCA_TENSORIZED_PROBE=0`` disables it.

    The published objects may be in CoreWeave's tensorizer wire format, which this
    framework does not read (parity unpinned: not in the tree): an object without the
    ``.tensors`` magic logs a warning and returns None, so the caller falls back to
    ``--model`` exactly as the reference's ``except OSError: pass`` does."""
    if os.environ.get("KCA_TENSORIZED_PROBE", "1") in ("0", "false", "no"):
        return None
    model_id = "/".join(model.rstrip("/").split("/")[-2:])
    base = os.environ.get("KCA_TENSORIZED_BASE", PUBLIC_TENSORIZED).rstrip("/")
    if not exists(f"{base}/{model_id}/model.tensors", timeout_s):
        return None
    sub = "fp16/" if fp16 else ""
    probe = f"{base}/{model_id}/{sub}model.tensors"
    if not is_kca_object(probe, timeout_s):
        import logging
        logging.getLogger(__name__).warning(
            "%s exists but is not a kca .tensors object (foreign tensorizer format?): loading --model instead",
            probe)
        return None
    if base == PUBLIC_TENSORIZED:
        return f"s3://tensorized/{model_id}/{sub}model.tensors"
    return probe


__all__ = ["Remote", "is_remote", "resolve", "exists", "is_kca_object", "read_header", "stream", "get_range",
           "public_tensorized_uri"]
