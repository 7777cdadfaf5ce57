"""KServe-compatible model server (V1 + V2 REST) on FastAPI/uvicorn.

The reference predictors subclass ``kserve.Model`` / ``kfserving.KFModel`` and
call ``ModelServer().start([model])`` (stable-diffusion/service/service.py:
135-270, bloom-176b/model/bloom.py:35-97, tensorizer-isvc kserve_api.py:18-78,
custom-sentiment/custom-predictor/model.py:6-30, gpt-2/transformer/
transformer.py:9-20). kserve is not part of this stack, so this module provides
the same contract natively:

* ``Model``: ``load`` / ``preprocess`` / ``predict`` / ``postprocess`` (sync or
  async), ``ready``; ``predictor_host`` turns it into a KServe *transformer*
  that forwards the preprocessed payload to the predictor's V1 endpoint;
  ``infer`` implements the V2 tensor protocol (Triton-compatible).
* ``ModelServer``: ``GET /``, ``GET /v1/models``, ``GET /v1/models/<m>``,
  ``POST /v1/models/<m>:predict``; ``GET /v2``, ``/v2/health/{live,ready}``,
  ``GET /v2/models/<m>[/versions/<v>][/ready]``, ``POST .../infer`` (JSON and
  the binary-tensor extension); Prometheus ``/metrics``. CLI flags as kserve's
  (``--http_port``, ``--grpc_port``, ``--workers``); default ports 8080 / 8081.
* the V2 gRPC service (``serving.grpc_v2``: ``GRPCInferenceService`` incl. the
  bidirectional ``ModelStreamInfer``) on ``--grpc_port`` for the same models.
"""
from __future__ import annotations

import argparse
import asyncio
import inspect
import logging
import os
import sys
import time

from fastapi import Request
from fastapi.responses import JSONResponse, Response

from . import v2

# GIL hand-off interval of the serving process. The engine's step loop runs in its own thread and gives
# the interpreter lock up at every device wait; under the default 5 ms interval, a request thread busy
# in JSON / tokenizer work can hold the engine off for up to 5 ms per hand-off (bench/serving_bench.py
# --switch-interval A/B)
GIL_SWITCH_S = 5e-4
# KCA_HTTP_FRONTEND=inline: the REST app in the engine's process (the default runs it in a child process
# whose models forward to this one: serving/frontend.py)
HTTP_FRONTEND = os.environ.get("KCA_HTTP_FRONTEND", "process")

log = logging.getLogger("kca.serving")


class InvalidInput(ValueError):
    pass


class Model:
    def __init__(self, name: str, predictor_host: str | None = None):
        self.name = name
        self.ready = False
        self.predictor_host = predictor_host

    def load(self):
        self.ready = True
        return self.ready

    def preprocess(self, payload, headers: dict | None = None):
        return payload

    def predict(self, payload, headers: dict | None = None):
        if self.predictor_host:
            return self._forward(payload)
        raise NotImplementedError

    def postprocess(self, result, headers: dict | None = None):
        return result

    # V2 tensor protocol (Triton-compatible); inputs/outputs are numpy arrays
    def infer(self, inputs: dict, request: dict, headers: dict | None = None) -> dict:
        raise NotImplementedError

    def metadata(self) -> dict:
        return {"name": self.name, "versions": ["1"], "platform": "kubernetes-cloud-amd", "inputs": [],
                "outputs": []}

    def _forward(self, payload):
        import httpx
        host = self.predictor_host
        if not host.startswith("http"):
            host = "http://" + host
        r = httpx.post(f"{host}/v1/models/{self.name}:predict", json=payload, timeout=600.0)
        r.raise_for_status()
        return r.json()

    async def __call__(self, payload, headers: dict | None = None):
        """preprocess -> predict -> postprocess. A sync stage runs on the event loop's executor; the
        base class's identity pre/postprocess are skipped, and a predictor with an async
        ``apredict`` (the continuous-batching text predictors: submit to the engine, await its
        future) holds no executor thread while it generates -- with every request parked in a
        blocking ``predict``, 32 in flight exhausted the executor and queued the next requests'
        pre/postprocess behind them (+143 ms p50 at concurrency 32, bench/serving_bench.py)."""
        async def run(fn, *a):
            if inspect.iscoroutinefunction(fn):
                return await fn(*a)
            return await asyncio.get_running_loop().run_in_executor(None, lambda: fn(*a))
        cls = type(self)
        x = payload if cls.preprocess is Model.preprocess else await run(self.preprocess, payload, headers)
        apredict = getattr(self, "apredict", None)
        y = await apredict(x, headers) if apredict is not None else await run(self.predict, x, headers)
        return y if cls.postprocess is Model.postprocess else await run(self.postprocess, y, headers)


def parse_server_args(argv=None):
    ap = argparse.ArgumentParser(add_help=False)
    ap.add_argument("--http_port", "--http-port", type=int, default=int(os.getenv("HTTP_PORT", 8080)))
    ap.add_argument("--grpc_port", "--grpc-port", type=int, default=8081)
    ap.add_argument("--workers", type=int, default=1)
    ap.add_argument("--host", default="0.0.0.0")
    args, _ = ap.parse_known_args(argv)
    return args


class ModelServer:
    def __init__(self, http_port: int | None = None, workers: int = 1, host: str | None = None,
                 argv: list | None = None):
        a = parse_server_args(argv)
        self.grpc_port = a.grpc_port
        self.http_port = http_port or a.http_port
        self.workers = workers or a.workers
        self.host = host or a.host
        self.models: dict = {}

    def register(self, model: Model):
        self.models[model.name] = model

    def create_app(self, models: list | None = None):
        from fastapi import FastAPI
        from fastapi.middleware.cors import CORSMiddleware
        from prometheus_client import CONTENT_TYPE_LATEST, CollectorRegistry, Counter, Histogram, generate_latest

        for m in models or []:
            self.register(m)
        if GIL_SWITCH_S > 0:
            sys.setswitchinterval(GIL_SWITCH_S)
        app = FastAPI(title="kubernetes-cloud-amd model server")
        app.add_middleware(CORSMiddleware, allow_origins=["*"], allow_methods=["*"], allow_headers=["*"])
        reg = CollectorRegistry()
        n_req = Counter("request_count", "requests", ["model", "protocol", "status"], registry=reg)
        lat = Histogram("request_latency_seconds", "latency", ["model", "protocol"], registry=reg,
                        buckets=(.005, .01, .025, .05, .1, .25, .5, 1, 2.5, 5, 10, 30, 60, 120))

        def get(name):
            m = self.models.get(name)
            if m is None:
                return None, JSONResponse({"error": f"Model with name {name} does not exist."}, status_code=404)
            if not m.ready:
                return None, JSONResponse({"error": f"Model with name {name} is not ready."}, status_code=503)
            return m, None

        @app.get("/")
        def live():
            return {"status": "alive"}

        @app.get("/metrics")
        def metrics():
            return Response(generate_latest(reg), media_type=CONTENT_TYPE_LATEST)

        @app.get("/v1/models")
        def list_models():
            return {"models": list(self.models)}

        @app.get("/v1/models/{name}")
        def model_ready(name: str):
            m = self.models.get(name)
            if m is None:
                return JSONResponse({"error": f"Model with name {name} does not exist."}, status_code=404)
            return JSONResponse({"name": name, "ready": bool(m.ready)}, status_code=200 if m.ready else 503)

        @app.post("/v1/models/{name}:predict")
        async def predict(name: str, request: Request):
            m, err = get(name)
            if err is not None:
                return err
            t0 = time.perf_counter()
            try:
                body = await request.body()
                import json
                payload = json.loads(body) if body else {}
                res = await m(payload, dict(request.headers))
            except (InvalidInput, ValueError, KeyError, TypeError) as e:
                n_req.labels(name, "v1", "400").inc()
                return JSONResponse({"error": str(e)}, status_code=400)
            except Exception as e:  # noqa: BLE001
                log.exception("predict failed")
                n_req.labels(name, "v1", "500").inc()
                return JSONResponse({"error": str(e)}, status_code=500)
            lat.labels(name, "v1").observe(time.perf_counter() - t0)
            n_req.labels(name, "v1", "200").inc()
            if isinstance(res, (bytes, bytearray)):
                mt = "image/png" if bytes(res[:8]) == b"\x89PNG\r\n\x1a\n" else "application/octet-stream"
                return Response(bytes(res), media_type=mt)
            if isinstance(res, Response):
                return res
            return JSONResponse(res)

        @app.get("/v2")
        def server_meta():
            return {"name": "kubernetes-cloud-amd", "version": "0.1", "extensions": ["binary_tensor_data"]}

        @app.get("/v2/health/live")
        def v2_live():
            return Response(status_code=200)

        @app.get("/v2/health/ready")
        def v2_ready():
            ok = all(m.ready for m in self.models.values())
            return Response(status_code=200 if ok else 503)

        @app.get("/v2/models/{name}")
        @app.get("/v2/models/{name}/versions/{version}")
        def v2_meta(name: str, version: str | None = None):
            m = self.models.get(name)
            if m is None:
                return JSONResponse({"error": f"Model with name {name} does not exist."}, status_code=404)
            return m.metadata()

        @app.get("/v2/models/{name}/ready")
        @app.get("/v2/models/{name}/versions/{version}/ready")
        def v2_model_ready(name: str, version: str | None = None):
            m = self.models.get(name)
            return Response(status_code=200 if (m is not None and m.ready) else 503)

        @app.post("/v2/models/{name}/infer")
        @app.post("/v2/models/{name}/versions/{version}/infer")
        async def v2_infer(name: str, request: Request, version: str | None = None):
            m, err = get(name)
            if err is not None:
                return err
            t0 = time.perf_counter()
            body = await request.body()
            hl = request.headers.get(v2.HEADER)
            try:
                req, inputs = v2.decode_request(body, int(hl) if hl else None)
                outs = await asyncio.get_running_loop().run_in_executor(
                    None, lambda: m.infer(inputs, req, dict(request.headers)))
                data, hdrs = v2.encode_response(name, outs, req, version or "1")
            except (InvalidInput, ValueError, KeyError, TypeError) as e:
                n_req.labels(name, "v2", "400").inc()
                return JSONResponse({"error": str(e)}, status_code=400)
            except Exception as e:  # noqa: BLE001
                log.exception("infer failed")
                n_req.labels(name, "v2", "500").inc()
                return JSONResponse({"error": str(e)}, status_code=500)
            lat.labels(name, "v2").observe(time.perf_counter() - t0)
            n_req.labels(name, "v2", "200").inc()
            mt = "application/octet-stream" if hdrs else "application/json"
            return Response(data, media_type=mt, headers=hdrs)

        return app

    def start(self, models: list, extra_routes=None):
        """``extra_routes(app)`` registers additional (non-KServe) routes, e.g.
        the bloom-inference-server API of ``serving.bloom_server``."""
        import uvicorn
        app = self.create_app(models)
        if extra_routes is not None:
            extra_routes(app)
        self.grpc_server = None
        if self.grpc_port and self.grpc_port > 0 and os.getenv("KCA_GRPC", "1") != "0":
            # KServe V2 / Triton GRPCInferenceService (incl. ModelStreamInfer) on the same models
            from .grpc_v2 import serve
            self.grpc_server = serve(self.models, self.grpc_port, self.host)
        log.info("serving %s on %s:%d", list(self.models), self.host, self.http_port)
        try:
            if HTTP_FRONTEND == "process" and extra_routes is None:
                # the REST stack in a child process, the engine's interpreter lock left to the engine
                # (serving/frontend.py)
                from .frontend import FrontendServer
                fe = FrontendServer(list(self.models.values()), self.http_port, self.host)
                try:
                    fe.wait()  # any front-end process dying ends the server (the pod restarts it)
                finally:
                    fe.close()
            else:
                uvicorn.run(app, host=self.host, port=self.http_port, workers=1, log_level="info")
        finally:
            if self.grpc_server is not None:
                self.grpc_server.stop(grace=2)


__all__ = ["Model", "ModelServer", "InvalidInput", "parse_server_args"]
