"""The REST front-end in processes of its own (serving/frontend.py, three sharing the port): V1 predict,
V2 infer and metadata through the proxy models, the model's errors mapped to the same status codes as
in process, and concurrent requests answered in any order."""
import socket
from concurrent.futures import ThreadPoolExecutor

import httpx
import numpy as np

from kubernetes_cloud_amd.serving.frontend import FrontendServer
from kubernetes_cloud_amd.serving.server import InvalidInput, Model


class Echo(Model):
    def __init__(self):
        super().__init__("echo")
        self.ready = True

    async def apredict(self, payload, headers=None):
        if "instances" not in payload:
            raise InvalidInput("request must contain 'instances'")
        if payload["instances"] == ["boom"]:
            raise RuntimeError("model failed")
        return {"predictions": [s[::-1] for s in payload["instances"]]}

    def infer(self, inputs, request, headers=None):
        return {"y": np.asarray(inputs["x"]) * 2}

    def metadata(self):
        return {"name": "echo", "versions": ["1"], "platform": "test", "inputs": [], "outputs": []}


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_frontend_process_routes_errors_and_concurrency():
    port = _port()
    fe = FrontendServer([Echo()], port, workers=3)
    try:
        base = f"http://127.0.0.1:{port}"
        r = httpx.post(f"{base}/v1/models/echo:predict", json={"instances": ["abc", "xyz"]})
        assert r.status_code == 200 and r.json() == {"predictions": ["cba", "zyx"]}
        assert httpx.post(f"{base}/v1/models/echo:predict", json={"nope": 1}).status_code == 400
        assert httpx.post(f"{base}/v1/models/echo:predict", json={"instances": ["boom"]}).status_code == 500
        assert httpx.post(f"{base}/v1/models/other:predict", json={"instances": []}).status_code == 404
        assert httpx.get(f"{base}/v2/models/echo").json()["platform"] == "test"
        body = {"inputs": [{"name": "x", "shape": [3], "datatype": "FP32", "data": [1.0, 2.0, 3.0]}]}
        out = httpx.post(f"{base}/v2/models/echo/infer", json=body).json()
        assert out["outputs"][0]["data"] == [2.0, 4.0, 6.0]
        words = [f"w{i:03d}" for i in range(48)]
        with ThreadPoolExecutor(16) as ex:  # new connections: spread over the three front-end processes
            got = list(ex.map(lambda w: httpx.post(f"{base}/v1/models/echo:predict",
                                                   json={"instances": [w]}).json()["predictions"][0], words))
        assert got == [w[::-1] for w in words]
    finally:
        fe.close()
    assert len(fe.procs) == 3 and all(p.poll() is not None for p in fe.procs)


def test_frontend_readiness_follows_engine_model_and_dead_worker_ends_wait():
    """the proxies report the engine-side model's readiness (not a constant True), and
    FrontendServer.wait() returns when ANY front-end process dies."""
    import time

    port = _port()
    m = Echo()
    m.ready = False
    fe = FrontendServer([m], port, workers=2)
    try:
        base = f"http://127.0.0.1:{port}"
        assert httpx.get(f"{base}/v2/models/echo/ready").status_code != 200
        m.ready = True
        time.sleep(1.2)  # the proxy re-asks after its TTL
        ok = [httpx.get(f"{base}/v2/models/echo/ready").status_code for _ in range(4)]
        assert all(c == 200 for c in ok), ok
        fe.procs[1].kill()
        t0 = time.time()
        rc = fe.wait()
        assert rc is not None and time.time() - t0 < 10
    finally:
        fe.close()
