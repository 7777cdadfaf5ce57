"""P2-P4 platform manifests and the img2dataset-compatible downloader."""
import http.server
import io
import json
import tarfile
import threading

import pyarrow as pa
import pyarrow.parquet as pq
from PIL import Image

from kubernetes_cloud_amd.data.img2dataset import download
from kubernetes_cloud_amd.deploy import platform


def test_dev_ssh_persists_root_and_requests_amd_gpus():
    m = platform.dev_ssh()
    dep = m["sshd-deployment.yaml"]["spec"]["template"]["spec"]
    c = dep["containers"][0]
    assert c["resources"]["limits"]["amd.com/gpu"] == 6
    sub = {v["subPath"] for v in c["volumeMounts"] if v.get("subPath")}
    assert {"etc", "usr", "home", "root"} <= sub
    assert "cp -ax / /target" in dep["initContainers"][0]["args"][0]
    assert m["sshd-service.yaml"]["spec"]["ports"][0]["port"] == 22


def test_jupyter_and_spark_manifests():
    j = platform.jupyter()
    c = j["jupyter-deployment.yaml"]["spec"]["template"]["spec"]["containers"][0]
    assert c["resources"]["limits"]["amd.com/gpu"] == 2 and c["ports"][0]["containerPort"] == 8888
    s = platform.spark()
    kinds = [d["kind"] for d in s["spark-role.yaml"]]
    assert kinds == ["ServiceAccount", "Role", "RoleBinding"]
    tpl = s["cpu-pod-template.yaml"]["spec"]
    assert "amd.com/gpu" not in json.dumps(tpl)  # CPU-only executors
    assert tpl["volumes"][0]["persistentVolumeClaim"]["claimName"] == "spark-pvc"


class _Img(http.server.BaseHTTPRequestHandler):
    def do_GET(self):  # noqa: N802
        if self.path.startswith("/missing"):
            self.send_response(404)
            self.end_headers()
            return
        buf = io.BytesIO()
        Image.new("RGB", (64, 32), (200, 10, 10)).save(buf, format="PNG")
        self.send_response(200)
        self.send_header("Content-Type", "image/png")
        self.end_headers()
        self.wfile.write(buf.getvalue())

    def log_message(self, *a):
        pass


def test_img2dataset_webdataset_shards(tmp_path):
    srv = http.server.ThreadingHTTPServer(("127.0.0.1", 0), _Img)
    th = threading.Thread(target=srv.serve_forever, daemon=True)
    th.start()
    try:
        base = f"http://127.0.0.1:{srv.server_address[1]}"
        urls = [f"{base}/img{i}.png" for i in range(5)] + [f"{base}/missing.png"]
        caps = [f"caption {i}" for i in range(6)]
        pq.write_table(pa.table({"URL": urls, "TEXT": caps}), tmp_path / "list.parquet")
        stats = download(str(tmp_path / "list.parquet"), str(tmp_path / "out"), thread_count=4,
                         image_size=32, subjob_size=4, processes=1)
    finally:
        srv.shutdown()
    assert [s["count"] for s in stats] == [4, 2]
    assert sum(s["successes"] for s in stats) == 5 and sum(s["failed_to_download"] for s in stats) == 1
    with tarfile.open(tmp_path / "out" / "00000.tar") as t:
        names = t.getnames()
        assert "000000000.jpg" in names and "000000000.txt" in names
        im = Image.open(t.extractfile("000000000.jpg"))
        assert im.size == (32, 32)
        assert t.extractfile("000000001.txt").read().decode() == "caption 1"
