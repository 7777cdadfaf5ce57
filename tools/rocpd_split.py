#!/usr/bin/env python3
"""Per-kernel split of the last N steps of a rocprofv3 trace database (``*_results.db``, the rocpd
SQLite output of ``rocprofv3 --kernel-trace``): a step ends at each dispatch of ``--step-kernel``.

    python tools/rocpd_split.py gpurun_out/prof/run_results.db --last-steps 10 --step-kernel sample_
Prints one line per (kernel, grid): calls per step, us per step, % of the step's busy time, then the
step's wall span (first start -> last end) and the gap time between kernels.
"""
from __future__ import annotations

import argparse
import collections
import sqlite3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--last-steps", type=int, default=10)
    ap.add_argument("--step-kernel", default="sample_")
    ap.add_argument("--top", type=int, default=30)
    a = ap.parse_args()
    c = sqlite3.connect(a.db)
    rows = c.execute("select name, start, end, grid_x, grid_y, workgroup_x from kernels order by start").fetchall()
    marks = [i for i, r in enumerate(rows) if a.step_kernel in r[0]]
    if len(marks) > a.last_steps:
        lo = marks[-a.last_steps - 1] + 1
    else:
        lo = 0
    rows = rows[lo:marks[-1] + 1] if marks else rows
    steps = min(a.last_steps, len(marks)) or 1
    agg = collections.defaultdict(lambda: [0, 0.0])
    busy = 0.0
    for name, s, e, gx, gy, wx in rows:
        key = (name.split("(")[0][:90], gx // max(wx, 1), gy)
        agg[key][0] += 1
        agg[key][1] += (e - s) / 1e3
        busy += (e - s) / 1e3
    span = (rows[-1][2] - rows[0][1]) / 1e3 if rows else 0.0
    print(f"steps {steps}: span/step {span / steps:.1f} us, kernel busy/step {busy / steps:.1f} us, "
          f"gaps/step {(span - busy) / steps:.1f} us, kernels/step {len(rows) / steps:.1f}")
    for (name, g, gy), (n, t) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:a.top]:
        print(f"{t / steps:9.1f} us {100 * t / busy:5.1f}%  x{n / steps:6.1f}  grid {g}x{gy}  {name}")


if __name__ == "__main__":
    main()
