"""StepWatchdog and tracing hooks."""
import json
import os
import subprocess
import sys
import time

from kubernetes_cloud_amd.obs.trace import mark, trace_range
from kubernetes_cloud_amd.utils.watchdog import StepWatchdog


def test_watchdog_fires_without_beats(tmp_path):
    hits = []
    wd = StepWatchdog(0.3, rank=3, report_dir=str(tmp_path), abort=False, poll_s=0.05,
                      on_timeout=lambda w: hits.append(w))
    with wd:
        wd.beat(7)
        deadline = time.time() + 5
        while not hits and time.time() < deadline:
            time.sleep(0.05)
    assert wd.fired and hits
    rep = json.loads((tmp_path / "watchdog-rank3.json").read_text())
    assert rep["last_step"] == 7 and rep["seconds_since_beat"] >= 0.3 and rep["stacks"]


def test_watchdog_quiet_while_beating(tmp_path):
    wd = StepWatchdog(0.5, report_dir=str(tmp_path), abort=False, poll_s=0.05)
    with wd:
        for i in range(20):
            wd.beat(i)
            time.sleep(0.05)
    assert not wd.fired
    assert not (tmp_path / "watchdog-rank0.json").exists()


def test_watchdog_abort_exit_code(tmp_path):
    code = ("import time; from kubernetes_cloud_amd.utils.watchdog import StepWatchdog;"
            f"StepWatchdog(0.5, report_dir={str(tmp_path)!r}, poll_s=0.05).start(); time.sleep(30)")
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    r = subprocess.run([sys.executable, "-c", code], cwd=root, env=dict(os.environ, PYTHONPATH=root),
                       capture_output=True, text=True, timeout=60)
    assert r.returncode == 124, r.stderr
    assert (tmp_path / "watchdog-rank0.json").exists()


def test_from_env(monkeypatch, tmp_path):
    monkeypatch.delenv("KCA_WATCHDOG_TIMEOUT", raising=False)
    assert StepWatchdog.from_env() is None
    monkeypatch.setenv("KCA_WATCHDOG_TIMEOUT", "12")
    monkeypatch.setenv("KCA_WATCHDOG_ABORT", "0")
    wd = StepWatchdog.from_env(rank=2, report_dir=str(tmp_path))
    assert wd.timeout_s == 12 and not wd.abort and wd.rank == 2


def test_trace_ranges_are_safe_without_a_profiler():
    with trace_range("outer"):
        with trace_range("inner"):
            mark("point")


def test_watchdog_adaptive_deadline(tmp_path):
    """factor x slowest step (after 2 beats); startup grace before the first beat."""
    import time as _t
    wd = StepWatchdog(0.1, report_dir=str(tmp_path), abort=False, poll_s=0.02, factor=4, startup_s=5)
    assert wd.deadline_s == 5  # no beat yet: startup grace
    wd.start()
    _t.sleep(0.3)  # a slow first step (startup) does not trip it
    assert not wd.fired
    wd.beat(1)
    _t.sleep(0.15)
    wd.beat(2)  # slowest step so far: 0.15 s -> deadline 0.6 s
    assert 0.55 < wd.deadline_s < 0.8
    _t.sleep(0.4)
    assert not wd.fired
    wd.beat(3)  # slowest step now ~0.4 s -> deadline ~1.6 s
    _t.sleep(2.5)  # a step 4x+ longer than any before -> fires
    assert wd.fired
    wd.stop()
