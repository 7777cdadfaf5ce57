#!/usr/bin/env python3
"""Per-kernel split of a window of optimizer steps in a rocprofv3 kernel trace: the steps are
delimited by the Nth..Mth calls of a marker kernel (default adamw_kernel, one per step), so a
trace that also holds other phases (bench.py secondaries) can be cut to the GPT-J steps.

    python tools/step_window.py gpurun_out/step_prof/step_kernel_trace.csv --first 2 --last 5
    (steps between the 2nd and 5th adamw calls = warmup 2, steps 3)
"""
import argparse
import collections
import csv
import re


def short(name: str) -> str:
    name = name.replace("(anonymous namespace)::", "")
    if name.startswith("void "):
        name = name[5:]
    depth, cut = 0, len(name)
    for i, ch in enumerate(name):  # drop the argument list, keep template arguments
        if ch == "<":
            depth += 1
        elif ch == ">":
            depth -= 1
        elif ch == "(" and depth == 0:
            cut = i
            break
    name = name[:cut]
    if name.startswith("Cijk_") or name.startswith("Custom_Cijk"):
        m = re.search(r"MT\d+x\d+x\d+", name)
        return "hipBLASLt " + (m.group(0) if m else name[:40])
    if "at::native" in name:
        m = re.search(r"at::native::(?:\(anonymous namespace\)::)?(\w+)", name)
        return "at::native::" + (m.group(1) if m else "?")
    return name[:90]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--marker", default="adamw_kernel")
    ap.add_argument("--first", type=int, default=2, help="window starts after this marker call (1-based)")
    ap.add_argument("--last", type=int, default=5, help="window ends at the end of this marker call")
    ap.add_argument("--top", type=int, default=30)
    ap.add_argument("--md", default="")
    a = ap.parse_args()
    rows = []
    with open(a.trace) as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    rows.sort()
    marks = [r for r in rows if a.marker in r[2]]
    t0, t1 = marks[a.first - 1][1], marks[a.last - 1][1]
    steps = a.last - a.first
    win = [r for r in rows if r[0] >= t0 and r[1] <= t1]
    busy = collections.Counter()
    calls = collections.Counter()
    for s, e, n in win:
        busy[short(n)] += e - s
        calls[short(n)] += 1
    tot = sum(busy.values())
    span = (t1 - t0) / steps / 1e3
    out = [f"steps {steps}  span/step {span:.1f} us  kernel-busy/step {tot / steps / 1e3:.1f} us",
           "| share | us/step | calls/step | kernel |", "|---|---|---|---|"]
    for k, v in busy.most_common(a.top):
        out.append(f"| {100 * v / tot:.2f}% | {v / steps / 1e3:.1f} | {calls[k] / steps:.0f} | `{k}` |")
    print("\n".join(out))
    if a.md:
        with open(a.md, "w") as f:
            f.write("\n".join(out) + "\n")


if __name__ == "__main__":
    main()
