"""Hang / failure detection for training and serving processes.

The reference delegates failure handling to Kubernetes, Argo and Knative
(retryStrategy, backoffLimit, restartPolicy: OnFailure, readiness probes --
finetuner-workflow/finetune-workflow.yaml:326-327, kubeflow/training-operator/
resnet50/k8s/imagenet-mpijob.yaml:12,63) and has no heartbeat or collective
timeout of its own: a rank stuck in an RCCL collective or a GPU fault that
wedges one process keeps the pod "Running" until the job deadline.

``StepWatchdog`` closes that gap for one process per GPU:

* the training loop calls ``beat(step)`` once per optimizer step;
* a daemon thread checks the age of the last beat; past ``timeout_s`` it
  writes a ``watchdog-rank{r}.json`` report (step, age, host, all thread
  stacks via ``faulthandler``) into ``report_dir`` and, when ``abort`` is set,
  terminates the process with exit code 124 so the pod's restartPolicy /
  Argo retryStrategy restarts it -- and the finetuner's checkpoint-N resume
  (finetuner.py:349-360 semantics) continues the run;
* RCCL's own async error handling is enabled (``TORCH_NCCL_ASYNC_ERROR_
  HANDLING=1``) so a collective that times out inside RCCL raises instead of
  blocking; ``init_distributed(timeout_s=...)`` carries the collective timeout.

Configuration from the environment (so manifests can set it without new CLI
flags): ``KCA_WATCHDOG_TIMEOUT`` seconds (0/unset = off), ``KCA_WATCHDOG_ABORT``
(default 1), ``KCA_WATCHDOG_DIR``, ``KCA_WATCHDOG_FACTOR`` (default 0 = off).

Adaptive deadline: with ``factor > 0`` the deadline is ``max(timeout_s, factor
x the slowest step seen so far)``, so a loaded node or a long first step
(graph capture, tuning, checkpoint write) never trips it while a step that
takes ``factor`` times longer than any before does; until the first beat the
deadline is ``max(timeout_s, startup_s)`` (``KCA_WATCHDOG_STARTUP``).
"""
from __future__ import annotations

import faulthandler
import io
import json
import os
import socket
import sys
import tempfile
import threading
import time


def enable_rccl_async_errors() -> None:
    os.environ.setdefault("TORCH_NCCL_ASYNC_ERROR_HANDLING", "1")
    os.environ.setdefault("TORCH_NCCL_BLOCKING_WAIT", "0")


class StepWatchdog:
    def __init__(self, timeout_s: float, rank: int = 0, report_dir: str | None = None,
                 abort: bool = True, poll_s: float | None = None, on_timeout=None, factor: float = 0.0,
                 startup_s: float = 0.0):
        self.timeout_s = float(timeout_s)
        self.factor = float(factor)
        self.startup_s = float(startup_s)
        self._max_step_s = 0.0
        self._beats = 0
        self.rank = rank
        self.report_dir = report_dir or tempfile.gettempdir()
        self.abort = abort
        self.poll_s = poll_s if poll_s is not None else max(0.05, min(5.0, self.timeout_s / 10))
        self.on_timeout = on_timeout
        self._last = time.monotonic()
        self._step = -1
        self._stop = threading.Event()
        self.fired = False
        self._thread: threading.Thread | None = None

    @classmethod
    def from_env(cls, rank: int = 0, report_dir: str | None = None) -> "StepWatchdog | None":
        t = float(os.environ.get("KCA_WATCHDOG_TIMEOUT", "0") or 0)
        if t <= 0:
            return None
        abort = os.environ.get("KCA_WATCHDOG_ABORT", "1") not in ("0", "false", "no")
        return cls(t, rank=rank, report_dir=os.environ.get("KCA_WATCHDOG_DIR", report_dir), abort=abort,
                   factor=float(os.environ.get("KCA_WATCHDOG_FACTOR", "0") or 0),
                   startup_s=float(os.environ.get("KCA_WATCHDOG_STARTUP", "0") or 0))

    def start(self) -> "StepWatchdog":
        enable_rccl_async_errors()
        self._last = time.monotonic()
        self._thread = threading.Thread(target=self._run, name="kca-watchdog", daemon=True)
        self._thread.start()
        return self

    def beat(self, step: int | None = None) -> None:
        now = time.monotonic()
        if self._beats:  # the first interval includes startup work: not a step time
            self._max_step_s = max(self._max_step_s, now - self._last)
        self._beats += 1
        self._last = now
        if step is not None:
            self._step = step

    @property
    def deadline_s(self) -> float:
        """Current allowed age of the last beat."""
        if self._beats == 0:
            return max(self.timeout_s, self.startup_s)
        if self.factor > 0 and self._beats >= 2:
            return max(self.timeout_s, self.factor * self._max_step_s)
        return max(self.timeout_s, self.startup_s) if self.factor > 0 else self.timeout_s

    def stop(self) -> None:
        self._stop.set()
        if self._thread is not None:
            self._thread.join(timeout=self.poll_s * 4)

    def __enter__(self):
        return self.start()

    def __exit__(self, *exc):
        self.stop()

    # ------------------------------------------------------------------
    def _stacks(self) -> str:
        buf = tempfile.TemporaryFile(mode="w+")
        try:
            faulthandler.dump_traceback(file=buf, all_threads=True)
            buf.seek(0)
            return buf.read()
        except (io.UnsupportedOperation, ValueError):  # pragma: no cover
            return ""
        finally:
            buf.close()

    def report(self, age: float) -> str:
        os.makedirs(self.report_dir, exist_ok=True)
        path = os.path.join(self.report_dir, f"watchdog-rank{self.rank}.json")
        rec = {"rank": self.rank, "host": socket.gethostname(), "pid": os.getpid(),
               "last_step": self._step, "seconds_since_beat": round(age, 3),
               "timeout_s": self.timeout_s, "deadline_s": round(self.deadline_s, 3),
               "max_step_s": round(self._max_step_s, 3), "time": time.time(), "stacks": self._stacks()}
        with open(path, "w") as f:
            json.dump(rec, f, indent=1)
        return path

    def _run(self):
        while not self._stop.wait(self.poll_s):
            age = time.monotonic() - self._last
            limit = self.deadline_s
            if age <= limit:
                continue
            self.fired = True
            path = self.report(age)
            print(f"[watchdog] rank {self.rank}: no step for {age:.1f}s (> {limit:.1f}s) after step "
                  f"{self._step}; report {path}", file=sys.stderr, flush=True)
            if self.on_timeout is not None:
                self.on_timeout(self)
            if self.abort:
                os._exit(124)
            return
