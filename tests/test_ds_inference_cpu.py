"""DeepSpeed-Inference pre-sharded BLOOM checkpoints (parallel/ds_inference_ckpt.py,
the microsoft/bloom-deepspeed-inference-fp16 layout of
bloom-176b-deepspeed/files/isvc-patch.txt:85-92): exported at tp_size 4 with 2
shards per rank, every TP shard rebuilt for world 1/2/4/8 must equal our own
shard of the full model. Also: the HF-snapshot downloader CLI and the S3
uploader (SigV4 PUTs, multipart) against a local server."""
import http.server
import json
import os
import threading

import pytest
import torch

from .helpers import make_model_dir


@pytest.fixture(scope="module")
def bloom(tmp_path_factory):
    from kubernetes_cloud_amd.io.hf import load_pretrained
    d = make_model_dir(str(tmp_path_factory.mktemp("bloom")), "bloom-560m", hidden_size=64, n_layer=2, n_head=8,
                       vocab_size=128, tokenizer=False)
    return d, load_pretrained(d, dtype=torch.float32)


@pytest.mark.parametrize("world", [1, 2, 4, 8])
def test_ds_inference_reshard(bloom, world, tmp_path):
    from kubernetes_cloud_amd.parallel.ds_inference_ckpt import export_ds_inference, is_ds_inference_dir, \
        load_ds_inference_tp
    from kubernetes_cloud_amd.parallel.tensor_parallel import shard_model_from_full
    d, full = bloom
    ck = export_ds_inference(d, str(tmp_path / "ds"), tp_size=4, shards_per_rank=2, dtype=torch.float32)
    assert is_ds_inference_dir(ck)
    cfgj = json.load(open(os.path.join(ck, "ds_inference_config.json")))
    assert cfgj["tp_size"] == 4 and len(cfgj["checkpoints"]["tp"]) == 8
    for rank in range(world):
        got = load_ds_inference_tp(ck, rank, world, dtype=torch.float32).state_dict()
        ref = shard_model_from_full(full, rank, world).state_dict()
        assert set(k for k in got if not k.endswith("alibi")) == set(k for k in ref if not k.endswith("alibi"))
        for k, v in ref.items():
            if k.endswith("alibi"):
                continue
            assert torch.equal(got[k], v), (world, rank, k)


def test_ds_inference_deepspeed_layout(bloom, tmp_path):
    """A hand-built checkpoint in DeepSpeed's own save layout: qkv
    entries as [tensor, dtype] lists, file names that carry no rank, ranks
    assigned by position in checkpoints.tp."""
    from kubernetes_cloud_amd.parallel.ds_inference_ckpt import export_ds_inference, load_ds_inference_tp
    from kubernetes_cloud_amd.parallel.tensor_parallel import shard_model_from_full
    d, full = bloom
    src = export_ds_inference(d, str(tmp_path / "ours"), tp_size=2, shards_per_rank=2, dtype=torch.float32)
    cfgj = json.load(open(os.path.join(src, "ds_inference_config.json")))
    out = tmp_path / "ds"
    out.mkdir()
    # DeepSpeed's TP save lists partition-major: [m0 r0, m0 r1, m1 r0, m1 r1]
    assert cfgj["checkpoints"]["tp"] == ["tp_00_00.pt", "tp_01_00.pt", "tp_00_01.pt", "tp_01_01.pt"]
    names = []
    for i, fn in enumerate(cfgj["checkpoints"]["tp"]):  # same positions, names without ranks
        sd = torch.load(os.path.join(src, fn), weights_only=True)
        sd = {k: ([v, "torch.float32"] if "query_key_value" in k else v) for k, v in sd.items()}
        name = f"bloom-ds-shard-{chr(ord('a') + i)}.pt"
        torch.save(sd, str(out / name))
        names.append(name)
    nt = torch.load(os.path.join(src, "non-tp.pt"), weights_only=True)
    torch.save(nt, str(out / "non-tp-weights.pt"))
    cfgj["checkpoints"] = {"non_tp": ["non-tp-weights.pt"], "tp": names}
    (out / "ds_inference_config.json").write_text(json.dumps(cfgj))
    (out / "config.json").write_text(open(os.path.join(src, "config.json")).read())
    for world in (1, 2):
        for rank in range(world):
            got = load_ds_inference_tp(str(out), rank, world, dtype=torch.float32).state_dict()
            ref = shard_model_from_full(full, rank, world).state_dict()
            for k, v in ref.items():
                if not k.endswith("alibi"):
                    assert torch.equal(got[k], v), (world, rank, k)


def test_hf_snapshot_cli_local_mirror(tmp_path, monkeypatch):
    """download.py contract (--model-id/--revision into $HF_HOME's hub cache), served
    here from a local mirror dir: the result resolves through the read-only
    refs -> snapshots layout the BLOOM DS server reads (isvc-patch.txt:55-77)."""
    from kubernetes_cloud_amd.data.hf_snapshot import main
    from kubernetes_cloud_amd.serving.bloom_server import resolve_hf_cache_path
    src = tmp_path / "mirror"
    src.mkdir()
    (src / "ds_inference_config.json").write_text("{}")
    monkeypatch.setenv("HF_HOME", str(tmp_path / "hf"))
    monkeypatch.setenv("KCA_HF_MIRROR", str(src))
    main(["--model-id=microsoft/bloom-deepspeed-inference-fp16", "--revision=main"])
    p = resolve_hf_cache_path("microsoft/bloom-deepspeed-inference-fp16", str(tmp_path / "hf" / "hub"))
    assert os.path.exists(os.path.join(p, "ds_inference_config.json"))


class _S3Handler(http.server.BaseHTTPRequestHandler):
    protocol_version = "HTTP/1.1"
    store: dict = {}
    auth: list = []
    parts: dict = {}

    def log_message(self, *a):
        pass

    def _body(self):
        n = int(self.headers.get("Content-Length", "0"))
        return self.rfile.read(n) if n else b""

    def _ok(self, data=b"", hdrs=None):
        self.send_response(200)
        for k, v in (hdrs or {}).items():
            self.send_header(k, v)
        self.send_header("Content-Length", str(len(data)))
        self.end_headers()
        self.wfile.write(data)

    def do_PUT(self):
        type(self).auth.append(self.headers.get("Authorization", ""))
        path, _, q = self.path.partition("?")
        body = self._body()
        if "partNumber" in q:
            num = int(q.split("partNumber=")[1].split("&")[0])
            type(self).parts.setdefault(path, {})[num] = body
            self._ok(hdrs={"ETag": f'"p{num}"'})
        else:
            type(self).store[path] = body
            self._ok(hdrs={"ETag": '"x"'})

    def do_POST(self):
        type(self).auth.append(self.headers.get("Authorization", ""))
        path, _, q = self.path.partition("?")
        self._body()
        if q.startswith("uploads"):
            self._ok(b"<InitiateMultipartUploadResult><UploadId>u1</UploadId></InitiateMultipartUploadResult>")
        else:
            parts = type(self).parts.pop(path)
            type(self).store[path] = b"".join(parts[i] for i in sorted(parts))
            self._ok(b"<CompleteMultipartUploadResult/>")


def test_s3_upload_recursive(tmp_path):
    from kubernetes_cloud_amd.io.s3_upload import S3, upload_tree

    class H(_S3Handler):
        store, auth, parts = {}, [], {}
    srv = http.server.ThreadingHTTPServer(("127.0.0.1", 0), H)
    threading.Thread(target=srv.serve_forever, daemon=True).start()
    src = tmp_path / "sd-model"
    (src / "unet").mkdir(parents=True)
    (src / "model_index.json").write_text("{}")
    big = os.urandom(3000)
    (src / "unet" / "unet.tensors").write_bytes(big)
    s3 = S3(f"http://127.0.0.1:{srv.server_address[1]}", "AK", "SK")
    keys = upload_tree(str(src), "s3://bucket/models", s3, acl_public=True, part_size=1024)
    srv.shutdown()
    assert sorted(keys) == ["models/sd-model/model_index.json", "models/sd-model/unet/unet.tensors"]
    assert H.store["/bucket/models/sd-model/unet/unet.tensors"] == big  # multipart, reassembled in order
    assert H.store["/bucket/models/sd-model/model_index.json"] == b"{}"
    assert all(a.startswith("AWS4-HMAC-SHA256 Credential=AK/") for a in H.auth)
