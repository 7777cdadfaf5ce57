"""Metrics sink: always a JSONL file, optionally Weights & Biases.

Metric names follow the reference (finetuner.py:516-532; sd-finetuner/
finetuner.py:562-598): ``perf/opt_time``, ``perf/gas_time``,
``perf/total_time_per_step``, ``perf/rank_samples_per_second``,
``perf/world_samples_per_second`` -- plus ``perf/tokens_per_second`` and
``perf/mfu``. W&B is used only when ``WANDB_API_KEY`` is set and the package
imports (the reference's rule, finetuner.py:364-393); otherwise disabled.
"""
from __future__ import annotations

import json
import os
import time


class MetricsSink:
    def __init__(self, log_dir: str, run_name: str, project: str = "kubernetes-cloud-amd",
                 enabled: bool = True, config: dict | None = None):
        self.enabled = enabled
        self.path = None
        self._wandb = None
        if not enabled:
            return
        os.makedirs(log_dir, exist_ok=True)
        self.path = os.path.join(log_dir, f"{run_name}.metrics.jsonl")
        self._f = open(self.path, "a", buffering=1)
        if os.environ.get("WANDB_API_KEY", "").strip():
            try:
                import wandb  # noqa: F401
                self._wandb = wandb.init(project=project, name=run_name, config=config or {},
                                         resume="allow")
            except Exception:
                self._wandb = None

    def log(self, metrics: dict, step: int | None = None):
        if not self.enabled:
            return
        rec = {"time": time.time(), "step": step, **metrics}
        self._f.write(json.dumps(rec, default=float) + "\n")
        if self._wandb is not None:
            try:
                self._wandb.log(metrics, step=step)
            except Exception:
                pass

    def close(self):
        if self.enabled:
            self._f.close()
            if self._wandb is not None:
                try:
                    self._wandb.finish()
                except Exception:
                    pass


class StepTimer:
    """Per-step phases, PerformanceCallback-style (gas = forward/backward of
    all micro-batches, opt = collectives + optimizer)."""

    def __init__(self, sync=None):
        self.sync = sync
        self.t0 = self.t_gas = None

    def start(self):
        if self.sync:
            self.sync()
        self.t0 = time.perf_counter()

    def gas_done(self):
        if self.sync:
            self.sync()
        self.t_gas = time.perf_counter()

    def stop(self, samples_per_rank: int, world: int, tokens_per_sample: int,
             flops_per_token: float | None = None, peak_flops: float = 2.5e15) -> dict:
        if self.sync:
            self.sync()
        t1 = time.perf_counter()
        total = t1 - self.t0
        rank_sps = samples_per_rank / total
        out = {
            "perf/opt_time": t1 - (self.t_gas or t1),
            "perf/gas_time": (self.t_gas or t1) - self.t0,
            "perf/total_time_per_step": total,
            "perf/rank_samples_per_second": rank_sps,
            "perf/world_samples_per_second": rank_sps * world,
            "perf/tokens_per_second": rank_sps * world * tokens_per_sample,
        }
        if flops_per_token:
            out["perf/mfu"] = rank_sps * tokens_per_sample * flops_per_token / peak_flops
        return out
