#!/usr/bin/env python3
"""rocprofv3 ``*_kernel_stats.csv`` -> markdown table (share, calls, avg us, kernel) with the eager
PyTorch (``at::native``) share and any softmax kernel called out.

    python tools/stats_md.py gpurun_out/sdt_prof_r4/sdt_kernel_stats.csv --title "..." --top 30
"""
import argparse
import csv


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("stats")
    ap.add_argument("--title", default="kernel split")
    ap.add_argument("--cmd", default="")
    ap.add_argument("--top", type=int, default=30)
    a = ap.parse_args()
    rows = list(csv.DictReader(open(a.stats)))
    tot = sum(float(r["TotalDurationNs"]) for r in rows)
    eager = sum(float(r["TotalDurationNs"]) for r in rows if "at::native" in r["Name"])
    soft = [r["Name"][:80] for r in rows if "softmax" in r["Name"].lower()]
    print(f"# {a.title}\n")
    if a.cmd:
        print(f"`{a.cmd}` (rocprofv3 --kernel-trace --stats; warm-up included).", end=" ")
    print(f"Total kernel time {tot / 1e6:.1f} ms; eager PyTorch (`at::native`) kernels **{100 * eager / tot:.2f} %**; "
          f"softmax kernels: {', '.join(soft) if soft else 'none'}.\n")
    print("| share | calls | avg us | kernel |\n|---|---|---|---|")
    for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:a.top]:
        print(f"| {100 * float(r['TotalDurationNs']) / tot:.2f}% | {r['Calls']} | {float(r['AverageNs']) / 1e3:.1f} | "
              f"`{r['Name'][:110]}` |")


if __name__ == "__main__":
    main()
