"""Recursive S3 upload (the stable-diffusion example's optional uploader job:
online-inference/stable-diffusion/03-optional-s3-upload-job.yaml:1-61 runs
``s3cmd put --recursive --acl-public <dir> s3://<bucket>/`` with keys from the
``s3-access-key`` / ``s3-secret-key`` / ``s3-host-url`` secrets).

    python -m kubernetes_cloud_amd.io.s3_upload --src /mnt/models/sd --dest s3://bucket/prefix [--acl-public]

Path-style PUTs signed with SigV4 (``UNSIGNED-PAYLOAD``, streamed from disk, no
whole-file buffering); credentials and endpoint from ``AWS_KEY``/``AWS_SECRET``/
``AWS_HOST`` (the reference job's env) or ``AWS_ACCESS_KEY_ID``/
``AWS_SECRET_ACCESS_KEY``/``S3_ENDPOINT_URL``. Objects larger than
``--part-size`` go up as an S3 multipart upload.
"""
from __future__ import annotations

import argparse
import datetime
import hashlib
import hmac
import http.client
import os
import re
import ssl
import sys
import urllib.parse
from xml.etree import ElementTree


def _sign(method: str, host: str, path: str, query: str, access: str, secret: str, region: str,
          extra: dict | None = None, now: datetime.datetime | None = None) -> dict:
    now = now or datetime.datetime.now(datetime.timezone.utc)
    amz = now.strftime("%Y%m%dT%H%M%SZ")
    day = amz[:8]
    hdrs = {"host": host, "x-amz-content-sha256": "UNSIGNED-PAYLOAD", "x-amz-date": amz}
    for k, v in (extra or {}).items():
        hdrs[k.lower()] = v
    names = sorted(hdrs)
    canon_q = "&".join(sorted(query.split("&"))) if query else ""
    canon = "\n".join([method, urllib.parse.quote(path, safe="/~"), canon_q,
                       "".join(f"{k}:{hdrs[k]}\n" for k in names), ";".join(names), "UNSIGNED-PAYLOAD"])
    scope = f"{day}/{region}/s3/aws4_request"
    sts = "\n".join(["AWS4-HMAC-SHA256", amz, scope, hashlib.sha256(canon.encode()).hexdigest()])

    def h(k, m):
        return hmac.new(k, m.encode(), hashlib.sha256).digest()
    key = h(h(h(h(("AWS4" + secret).encode(), day), region), "s3"), "aws4_request")
    sig = hmac.new(key, sts.encode(), hashlib.sha256).hexdigest()
    out = {k: v for k, v in hdrs.items() if k != "host"}
    out["Authorization"] = (f"AWS4-HMAC-SHA256 Credential={access}/{scope}, SignedHeaders={';'.join(names)}, "
                            f"Signature={sig}")
    return out


class S3:
    def __init__(self, endpoint: str, access: str, secret: str, region: str = "us-east-1",
                 verify: bool = True, timeout: float = 300.0):
        if "://" not in endpoint:
            endpoint = "https://" + endpoint
        u = urllib.parse.urlsplit(endpoint)
        self.tls = u.scheme == "https"
        self.host = u.hostname
        self.port = u.port or (443 if self.tls else 80)
        self.hosthdr = self.host if u.port in (None, 80, 443) else f"{self.host}:{self.port}"
        self.access, self.secret, self.region = access, secret, region
        self.verify, self.timeout = verify, timeout

    def _conn(self):
        if self.tls:
            ctx = ssl.create_default_context()
            if not self.verify:
                ctx.check_hostname = False
                ctx.verify_mode = ssl.CERT_NONE
            return http.client.HTTPSConnection(self.host, self.port, timeout=self.timeout, context=ctx)
        return http.client.HTTPConnection(self.host, self.port, timeout=self.timeout)

    def request(self, method: str, path: str, query: str = "", body=None, length: int | None = None,
                headers: dict | None = None) -> bytes:
        h = _sign(method, self.hosthdr, path, query, self.access, self.secret, self.region, headers)
        if length is not None:
            h["Content-Length"] = str(length)
        c = self._conn()
        try:
            c.request(method, urllib.parse.quote(path, safe="/~") + (f"?{query}" if query else ""), body=body,
                      headers=h)
            r = c.getresponse()
            data = r.read()
            if r.status >= 300:
                raise IOError(f"S3 {method} {path}: HTTP {r.status} {data[:300]!r}")
            return data, r
        finally:
            c.close()

    def put_file(self, local: str, bucket: str, key: str, acl_public: bool = False, part_size: int = 256 << 20):
        size = os.path.getsize(local)
        path = f"/{bucket}/{key}"
        extra = {"x-amz-acl": "public-read"} if acl_public else {}
        if size <= part_size:
            with open(local, "rb") as f:
                self.request("PUT", path, body=f, length=size, headers=extra)
            return
        data, _ = self.request("POST", path, "uploads=", headers=extra)
        upload_id = re.search(rb"<UploadId>([^<]+)</UploadId>", data).group(1).decode()
        etags = []
        with open(local, "rb") as f:
            for i, off in enumerate(range(0, size, part_size), start=1):
                n = min(part_size, size - off)
                f.seek(off)
                chunk = f.read(n)
                _, r = self.request("PUT", path, f"partNumber={i}&uploadId={urllib.parse.quote(upload_id)}",
                                    body=chunk, length=n)
                etags.append((i, r.getheader("ETag")))
        root = ElementTree.Element("CompleteMultipartUpload")
        for i, e in etags:
            p = ElementTree.SubElement(root, "Part")
            ElementTree.SubElement(p, "PartNumber").text = str(i)
            ElementTree.SubElement(p, "ETag").text = e
        xml = ElementTree.tostring(root)
        self.request("POST", path, f"uploadId={urllib.parse.quote(upload_id)}", body=xml, length=len(xml))


def upload_tree(src: str, dest: str, s3: S3, acl_public: bool = False, part_size: int = 256 << 20) -> list:
    """``s3cmd put --recursive src s3://bucket/prefix/``: the directory itself is
    uploaded under the prefix (``prefix/<basename(src)>/...``), like s3cmd."""
    if not dest.startswith("s3://"):
        raise ValueError("dest must be s3://bucket[/prefix]")
    bucket, _, prefix = dest[5:].partition("/")
    prefix = prefix.strip("/")
    base = os.path.basename(os.path.normpath(src))
    done = []
    for root, _, files in os.walk(src):
        for fn in sorted(files):
            local = os.path.join(root, fn)
            rel = os.path.relpath(local, src).replace(os.sep, "/")
            key = "/".join(x for x in (prefix, base, rel) if x)
            s3.put_file(local, bucket, key, acl_public, part_size)
            done.append(key)
    return done


def main(argv=None):
    ap = argparse.ArgumentParser(description="recursive S3 upload (s3cmd put --recursive)")
    ap.add_argument("--src", required=True)
    ap.add_argument("--dest", required=True, help="s3://bucket[/prefix]")
    ap.add_argument("--acl-public", action="store_true")
    ap.add_argument("--part-size", type=int, default=256 << 20)
    a = ap.parse_args(argv)
    env = os.environ
    access = env.get("AWS_KEY") or env.get("AWS_ACCESS_KEY_ID")
    secret = env.get("AWS_SECRET") or env.get("AWS_SECRET_ACCESS_KEY")
    host = env.get("AWS_HOST") or env.get("S3_ENDPOINT_URL") or "https://object.ord1.coreweave.com"
    if not access or not secret:
        print("missing credentials (AWS_KEY/AWS_SECRET)", file=sys.stderr)
        return 2
    s3 = S3(host, access, secret, env.get("AWS_DEFAULT_REGION", "us-east-1"),
            verify=env.get("KCA_TLS_VERIFY", "1") not in ("0", "false"))
    for k in upload_tree(a.src, a.dest, s3, a.acl_public, a.part_size):
        print(f"upload: s3://{a.dest[5:].partition('/')[0]}/{k}")
    return 0


if __name__ == "__main__":
    sys.exit(main())
