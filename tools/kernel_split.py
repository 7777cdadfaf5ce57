#!/usr/bin/env python3
"""Per-(kernel, grid) time split of a rocprofv3 kernel trace (``*_kernel_trace.csv``),
optionally restricted to the last N dispatches of a kernel that marks one step.

    python tools/kernel_split.py gpurun_out/dec_prof/dec_kernel_trace.csv --last-steps 30 --step-kernel sample_kernel
"""
import argparse
import collections
import csv


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--last-steps", type=int, default=0)
    ap.add_argument("--step-kernel", default="sample_kernel")
    ap.add_argument("--top", type=int, default=30)
    a = ap.parse_args()
    rows = sorted(csv.DictReader(open(a.trace)), key=lambda r: int(r["Start_Timestamp"]))
    if a.last_steps:
        marks = [i for i, r in enumerate(rows) if r["Kernel_Name"].startswith(a.step_kernel)]
        lo = marks[-a.last_steps - 1] + 1 if len(marks) > a.last_steps else 0
        rows = rows[lo:marks[-1] + 1]
        steps = a.last_steps
    else:
        steps = 1
    agg = collections.defaultdict(lambda: [0, 0.0])
    for r in rows:
        name = r["Kernel_Name"].split("(")[0][:70]
        key = (name, int(r["Grid_Size_X"]) // int(r["Workgroup_Size_X"]), r["Grid_Size_Y"], r["Grid_Size_Z"])
        agg[key][0] += 1
        agg[key][1] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    busy = sum(v[1] for v in agg.values())
    span = (int(rows[-1]["End_Timestamp"]) - int(rows[0]["Start_Timestamp"])) / 1e3
    print(f"steps {steps}  span/step {span / steps:.1f} us  kernel-busy/step {busy / steps:.1f} us  "
          f"gaps/step {(span - busy) / steps:.1f} us")
    print(f"{'us/step':>9} {'calls/step':>10} {'us/call':>8}  wgs(x,y,z)  kernel")
    for (name, gx, gy, gz), (n, t) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:a.top]:
        print(f"{t / steps:9.1f} {n / steps:10.2f} {t / n:8.2f}  {gx},{gy},{gz}  {name}")


if __name__ == "__main__":
    main()
