#!/usr/bin/env python3
"""Per-kernel stats of the steady-state part of a rocprofv3 kernel trace: the
dispatches after the last idle gap longer than 0.5 s (the benches sleep before their timed
loop), so one-time work such as MIOpen find or graph capture is excluded.

Usage: python tools/steady_stats.py <kernel_trace.csv> [--top 30] [--csv out.csv]
"""
import argparse
import csv
from collections import defaultdict

ap = argparse.ArgumentParser()
ap.add_argument("trace")
ap.add_argument("--top", type=int, default=30)
ap.add_argument("--csv")
a = ap.parse_args()
rows = sorted(csv.DictReader(open(a.trace)), key=lambda r: int(r["Start_Timestamp"]))
st = [int(r["Start_Timestamp"]) for r in rows]
gaps = [(st[i + 1] - int(rows[i]["End_Timestamp"]), i + 1) for i in range(len(rows) - 1)]
big = [i for g, i in gaps if g > 0.5e9]  # the benches sleep 1 s before each timed loop
cut = big[-1] if big else max(gaps)[1]
rows = rows[cut:]
agg = defaultdict(lambda: [0, 0])
for r in rows:
    d = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    agg[r["Kernel_Name"]][0] += 1
    agg[r["Kernel_Name"]][1] += d
tot = sum(v[1] for v in agg.values())
span = int(rows[-1]["End_Timestamp"]) - int(rows[0]["Start_Timestamp"])
print(f"steady dispatches {len(rows)}  kernel time {tot / 1e6:.2f} ms  span {span / 1e6:.2f} ms")
out = sorted(agg.items(), key=lambda kv: -kv[1][1])
for name, (n, t) in out[: a.top]:
    print(f"{n:6d} {t / n / 1e3:9.1f} us {100 * t / tot:6.2f}%  {name[:110]}")
if a.csv:
    with open(a.csv, "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage"])
        for name, (n, t) in out:
            w.writerow([name, n, t, t / n, 100 * t / tot])
