"""HTTP front-end in a process of its own (the KServe model server's HTTP stack beside the model).

The model server's REST app (``server.ModelServer.create_app``: uvicorn + FastAPI, request parsing,
JSON, routing, Prometheus metrics) is pure Python. Run in the process that owns the GPU engine, it
takes the interpreter lock for ~1.6 ms per request, and at 32 requests in flight that competes with
the continuous-batching loop that launches every decode step: the GPT-J predictor served 22 % fewer
requests/s over HTTP than through the same entry point in process (bench/serving_bench.py). Here the
HTTP app runs in a child process whose models are proxies; a proxy call sends (model, operation,
arguments) over a Unix-socket connection, and the engine process runs the real model's coroutine on
an event loop thread of its own and sends the result back -- its per-request Python is the pickle of
a small dict each way.

    srv = FrontendServer(models, port)   # engine process: starts the child, serves the calls
    ...
    srv.close()

Errors raised by the model (``InvalidInput``, ``ValueError`` ...) are re-raised in the front-end with
their type, so the REST layer maps them to the same status codes.
"""
from __future__ import annotations

import asyncio
import concurrent.futures
import itertools
import logging
import os
import secrets
import subprocess
import sys
import tempfile
import threading
import time

log = logging.getLogger(__name__)

# exception types carried across the connection by name (the REST layer's 400s, then any error)
_ERRORS = ("InvalidInput", "ValueError", "KeyError", "TypeError")


def _rebuild_error(kind: str, msg: str) -> Exception:
    from .server import InvalidInput
    return {"InvalidInput": InvalidInput, "ValueError": ValueError, "KeyError": KeyError,
            "TypeError": TypeError}.get(kind, RuntimeError)(msg)


class _Engine:
    """Engine-process side: one connection from the front-end; a reader thread, and the models'
    coroutines on an event loop thread."""

    def __init__(self, models: dict, conn):
        self.models, self.conn = models, conn
        self.send_lock = threading.Lock()
        self.loop = asyncio.new_event_loop()
        self.loop_th = threading.Thread(target=self.loop.run_forever, name="kca-engine-loop", daemon=True)
        self.loop_th.start()
        self.reader = threading.Thread(target=self._read, name="kca-frontend-reader", daemon=True)
        self.reader.start()

    def _send(self, msg):
        with self.send_lock:
            self.conn.send(msg)

    def _read(self):
        while True:
            try:
                msg = self.conn.recv()
            except (EOFError, OSError):
                return
            asyncio.run_coroutine_threadsafe(self._handle(*msg), self.loop)

    async def _handle(self, rid, name, op, args):
        try:
            m = self.models[name]
            if op == "call":
                res = await m(*args)
            elif op == "infer":
                res = await asyncio.get_running_loop().run_in_executor(None, lambda: m.infer(*args))
            else:
                raise ValueError(f"unknown operation {op}")
            self._send((rid, True, res))
        except Exception as e:  # noqa: BLE001 - every failure goes back to the waiting request
            kind = type(e).__name__
            self._send((rid, False, (kind if kind in _ERRORS else "RuntimeError", str(e))))

    def close(self):
        try:
            self.conn.close()
        except OSError:
            pass
        self.loop.call_soon_threadsafe(self.loop.stop)


class _Client:
    """Front-end side of the connection: requests tagged with ids, one reader thread resolving them."""

    def __init__(self, conn):
        self.conn = conn
        self.send_lock = threading.Lock()
        self.ids = itertools.count()
        self.pending: dict = {}
        threading.Thread(target=self._read, name="kca-frontend-client", daemon=True).start()

    def _read(self):
        while True:
            try:
                rid, ok, val = self.conn.recv()
            except (EOFError, OSError):
                for fut in list(self.pending.values()):
                    fut.set_exception(RuntimeError("engine process connection closed"))
                return
            fut = self.pending.pop(rid)
            if ok:
                fut.set_result(val)
            else:
                fut.set_exception(_rebuild_error(*val))

    def submit(self, name, op, *args) -> concurrent.futures.Future:
        fut: concurrent.futures.Future = concurrent.futures.Future()
        rid = next(self.ids)
        self.pending[rid] = fut
        with self.send_lock:
            self.conn.send((rid, name, op, args))
        return fut


def _proxy_models(client: _Client, meta: dict):
    from .server import Model

    class ProxyModel(Model):
        def __init__(self, name, md):
            super().__init__(name)
            self.ready, self._md = True, md

        async def __call__(self, payload, headers=None):
            return await asyncio.wrap_future(client.submit(self.name, "call", payload, headers))

        def infer(self, inputs, request, headers=None):
            return client.submit(self.name, "infer", inputs, request, headers).result()

        def metadata(self):
            return self._md

    return [ProxyModel(n, md) for n, md in meta.items()]


def _frontend_main():
    """Child process: connect back, build the proxies, serve the REST app."""
    from multiprocessing.connection import Client

    import uvicorn

    from .server import ModelServer
    addr, port, host = sys.argv[1], int(sys.argv[2]), sys.argv[3]
    key = bytes.fromhex(os.environ.pop("KCA_FRONTEND_KEY"))
    conn = Client(addr, family="AF_UNIX", authkey=key)
    meta = conn.recv()  # {name: metadata}
    client = _Client(conn)
    app = ModelServer(http_port=port, argv=[]).create_app(_proxy_models(client, meta))
    uvicorn.run(app, host=host, port=port, workers=1, log_level="warning", access_log=False)


class FrontendServer:
    """Engine process: start the front-end child on ``port`` and serve its model calls until
    ``close()`` (the constructor returns once the child answers its health route)."""

    def __init__(self, models: list, port: int, host: str = "127.0.0.1", start_timeout: float = 120.0):
        from multiprocessing.connection import Listener

        from . import server as _srv
        if _srv.GIL_SWITCH_S > 0:  # this process's threads (engine loop, model loop, reader) hand off often
            sys.setswitchinterval(_srv.GIL_SWITCH_S)
        self.port, self.host = port, host
        self.models = {m.name: m for m in models}
        d = tempfile.mkdtemp(prefix="kca_frontend_")
        self.addr = os.path.join(d, "sock")
        key = secrets.token_bytes(16)
        listener = Listener(self.addr, family="AF_UNIX", authkey=key)
        env = dict(os.environ, KCA_FRONTEND_KEY=key.hex(), CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="")
        root = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
        env["PYTHONPATH"] = root + os.pathsep + env.get("PYTHONPATH", "")
        self.proc = subprocess.Popen([sys.executable, "-m", "kubernetes_cloud_amd.serving.frontend", self.addr,
                                      str(port), host], env=env)
        got: list = []
        th = threading.Thread(target=lambda: got.append(listener.accept()), daemon=True)
        th.start()
        t0 = time.time()
        while th.is_alive():  # (accept has no timeout: watch the child instead)
            th.join(timeout=0.2)
            if self.proc.poll() is not None or time.time() - t0 > start_timeout:
                listener.close()
                self.proc.kill()
                raise RuntimeError("HTTP front-end did not connect")
        listener.close()
        conn = got[0]
        conn.send({n: m.metadata() for n, m in self.models.items()})
        self.engine = _Engine(self.models, conn)
        self._wait_ready(start_timeout)

    def _wait_ready(self, timeout: float):
        import httpx
        t0 = time.time()
        while time.time() - t0 < timeout:
            if self.proc.poll() is not None:
                raise RuntimeError(f"HTTP front-end exited with {self.proc.returncode}")
            try:
                if httpx.get(f"http://{self.host}:{self.port}/", timeout=2.0).status_code == 200:
                    return
            except httpx.HTTPError:
                pass
            time.sleep(0.1)
        raise RuntimeError("HTTP front-end did not start")

    def close(self):
        self.proc.terminate()
        try:
            self.proc.wait(timeout=30)
        except subprocess.TimeoutExpired:
            self.proc.kill()
            self.proc.wait(timeout=30)
        self.engine.close()
        try:
            os.unlink(self.addr)
            os.rmdir(os.path.dirname(self.addr))
        except OSError:
            pass


if __name__ == "__main__":
    _frontend_main()
