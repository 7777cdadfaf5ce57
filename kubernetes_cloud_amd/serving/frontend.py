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

    srv = FrontendServer(models, port)   # engine process: starts the children, serves the calls
    ...
    srv.close()

``workers`` front-end processes (KCA_HTTP_WORKERS, default 1) listen on the same port (SO_REUSEPORT:
the kernel spreads connections over them), each with its own connection to the engine process. GPT-J
at concurrency 32 served 121 req/s with 4 of them against 137 with one (bench/serving_bench.py,
round 5): the per-request work left at that load is in the engine process (result pickling, the
model coroutines' tokenisation, thread hand-offs), and more connections only add hand-offs there.

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
    """Engine-process side: one connection per front-end process, a reader thread each, and the
    models' coroutines on ONE event loop thread."""

    def __init__(self, models: dict, conns: list):
        self.models, self.conns = models, list(conns)
        self.send_locks = [threading.Lock() for _ in self.conns]
        self.loop = asyncio.new_event_loop()
        self.loop_th = threading.Thread(target=self.loop.run_forever, name="kca-engine-loop", daemon=True)
        self.loop_th.start()
        self.readers = [threading.Thread(target=self._read, args=(i,), name=f"kca-frontend-reader-{i}", daemon=True)
                        for i in range(len(self.conns))]
        for th in self.readers:
            th.start()

    def _send(self, i, msg):
        with self.send_locks[i]:
            self.conns[i].send(msg)

    def _read(self, i):
        while True:
            try:
                msg = self.conns[i].recv()
            except (EOFError, OSError):
                return
            asyncio.run_coroutine_threadsafe(self._handle(i, *msg), self.loop)

    async def _handle(self, i, rid, name, op, args):
        try:
            m = self.models[name]
            if op == "call":
                res = await m(*args)
            elif op == "ready":  # the front-end's health / readiness routes ask the real model
                res = bool(getattr(m, "ready", True))
            elif op == "infer":
                res = await asyncio.get_running_loop().run_in_executor(None, lambda: m.infer(*args))
            else:
                raise ValueError(f"unknown operation {op}")
            self._send(i, (rid, True, res))
        except Exception as e:  # noqa: BLE001 - every failure goes back to the waiting request
            kind = type(e).__name__
            try:
                self._send(i, (rid, False, (kind if kind in _ERRORS else "RuntimeError", str(e))))
            except OSError:  # that front-end process is gone
                pass

    def close(self):
        for c in self.conns:
            try:
                c.close()
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
        """The engine-side model seen from the front-end: calls go over the connection; ``ready`` is the
        real model's, asked again at most every READY_TTL_S seconds (a constant True kept
        /v2/health/ready and the model-ready routes green whatever the engine's model said)."""
        READY_TTL_S = 1.0

        def __init__(self, name, md):
            super().__init__(name)
            self._md = md
            self._ready_at, self._ready_val = 0.0, False

        @property
        def ready(self):
            now = time.monotonic()
            if now - self._ready_at > self.READY_TTL_S:
                try:
                    self._ready_val = bool(client.submit(self.name, "ready").result(timeout=5.0))
                except Exception:  # noqa: BLE001 - engine unreachable: not ready
                    self._ready_val = False
                self._ready_at = now
            return self._ready_val

        @ready.setter
        def ready(self, v):  # (Model.__init__ assigns it)
            self._ready_val = bool(v)

        async def __call__(self, payload, headers=None):
            return await asyncio.wrap_future(client.submit(self.name, "call", payload, headers))

        def infer(self, inputs, request, headers=None):
            return client.submit(self.name, "infer", inputs, request, headers).result()

        def metadata(self):
            return self._md

    return [ProxyModel(n, md) for n, md in meta.items()]


def _frontend_main():
    """Child process: connect back, build the proxies, listen on the shared port, serve the REST app."""
    import socket
    from multiprocessing.connection import Client

    import uvicorn

    from .server import ModelServer
    addr, port, host = sys.argv[1], int(sys.argv[2]), sys.argv[3]
    key = bytes.fromhex(os.environ.pop("KCA_FRONTEND_KEY"))
    conn = Client(addr, family="AF_UNIX", authkey=key)
    meta = conn.recv()  # {name: metadata}
    app = ModelServer(http_port=port, argv=[]).create_app(_proxy_models(_Client(conn), meta))
    fam = socket.AF_INET6 if ":" in host else socket.AF_INET
    # (proto given explicitly: asyncio sets TCP_NODELAY only on sockets whose proto is IPPROTO_TCP --
    # with proto 0 the accepted connections keep Nagle, +40 ms per response at concurrency 1)
    sock = socket.socket(fam, socket.SOCK_STREAM, socket.IPPROTO_TCP)
    sock.setsockopt(socket.SOL_SOCKET, socket.SO_REUSEADDR, 1)
    sock.setsockopt(socket.SOL_SOCKET, socket.SO_REUSEPORT, 1)
    sock.bind((host, port))
    sock.listen(2048)  # (connections queue here until the loop below runs)
    conn.send("listening")  # (before any request: the client's reader only receives)
    server = uvicorn.Server(uvicorn.Config(app, host=host, port=port, log_level="warning", access_log=False))
    server.run(sockets=[sock])


class FrontendServer:
    """Engine process: start ``workers`` front-end processes on ``port`` and serve their model calls
    until ``close()`` (the constructor returns once they listen and one answers the health route)."""

    def __init__(self, models: list, port: int, host: str = "127.0.0.1", start_timeout: float = 120.0,
                 workers: int | None = None):
        from multiprocessing.connection import Listener

        from . import server as _srv
        if _srv.GIL_SWITCH_S > 0:  # this process's threads (engine loop, model loop, readers) hand off often
            sys.setswitchinterval(_srv.GIL_SWITCH_S)
        self.port, self.host = port, host
        self.workers = max(1, int(os.environ.get("KCA_HTTP_WORKERS", "1")) if workers is None else int(workers))
        self.models = {m.name: m for m in models}
        d = tempfile.mkdtemp(prefix="kca_frontend_")
        self.addr = os.path.join(d, "sock")
        key = secrets.token_bytes(16)
        listener = Listener(self.addr, family="AF_UNIX", authkey=key, backlog=max(self.workers, 1))
        env = dict(os.environ, KCA_FRONTEND_KEY=key.hex(), CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="")
        root = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
        env["PYTHONPATH"] = root + os.pathsep + env.get("PYTHONPATH", "")
        self.procs = [subprocess.Popen([sys.executable, "-m", "kubernetes_cloud_amd.serving.frontend", self.addr,
                                        str(port), host], env=env) for _ in range(self.workers)]
        self.proc = self.procs[0]
        conns: list = []

        def accept_all():
            try:
                while len(conns) < self.workers:
                    conns.append(listener.accept())
            except OSError:  # listener closed by the watchdog below
                pass
        th = threading.Thread(target=accept_all, daemon=True)
        th.start()
        t0 = time.time()
        try:
            while th.is_alive():  # (accept has no timeout: watch the children instead)
                th.join(timeout=0.2)
                if any(p.poll() is not None for p in self.procs) or time.time() - t0 > start_timeout:
                    raise RuntimeError("HTTP front-end did not connect")
            meta = {n: m.metadata() for n, m in self.models.items()}
            for c in conns:
                c.send(meta)
            for c in conns:  # each child has bound and listens on the port
                if not c.poll(start_timeout) or c.recv() != "listening":
                    raise RuntimeError("HTTP front-end did not listen")
        except BaseException:
            listener.close()
            self._kill()
            raise
        listener.close()
        self.engine = _Engine(self.models, conns)
        self._wait_ready(start_timeout)

    def wait(self) -> int:
        """Block until ANY front-end process exits (watching only the first left a dead
        second worker unnoticed while its share of connections failed); the others are stopped.
        Returns that process's exit code."""
        while True:
            for p in self.procs:
                rc = p.poll()
                if rc is not None:
                    log.error("front-end process %d exited with %s; stopping the server", p.pid, rc)
                    return rc
            time.sleep(0.5)

    def _kill(self):
        for p in self.procs:
            if p.poll() is None:
                p.kill()

    def _wait_ready(self, timeout: float):
        import httpx
        t0 = time.time()
        while time.time() - t0 < timeout:
            dead = [p.returncode for p in self.procs if p.poll() is not None]
            if dead:
                raise RuntimeError(f"HTTP front-end exited with {dead[0]}")
            try:
                if httpx.get(f"http://{self.host}:{self.port}/", timeout=2.0).status_code == 200:
                    return
            except httpx.HTTPError:
                pass
            time.sleep(0.1)
        raise RuntimeError("HTTP front-end did not start")

    def close(self):
        for p in self.procs:
            p.terminate()
        for p in self.procs:
            try:
                p.wait(timeout=30)
            except subprocess.TimeoutExpired:
                p.kill()
                p.wait(timeout=30)
        self.engine.close()
        try:
            os.unlink(self.addr)
            os.rmdir(os.path.dirname(self.addr))
        except OSError:
            pass


if __name__ == "__main__":
    _frontend_main()
