#!/usr/bin/env python3
"""Per-mode sampler kernel time from a rocprofv3 kernel trace of tools/sample_bench.py.

    rocprofv3 --kernel-trace --output-format csv -d gpurun_out/samp -o s -- python3 tools/sample_bench.py
    python tools/sampler_profile.py gpurun_out/samp/s_kernel_trace.csv

Every ``kca_sample_logits`` call of the bench starts with sample_mwg_kernel (all its modes are
multi-workgroup rows), followed by the closing one-workgroup kernel (sample_reg_kernel / sample_kernel)
unless the caller passed mwg_complete (greedy / top-k rows, as the decode engine does); a call's time
is the sum of its kernels. sample_bench.py runs, per batch size, each mode 5 + 200 times in a fixed
order; the table gives the median over the 200 timed calls of each (batch, mode)."""
import csv
import statistics
import sys

MODES = ["greedy", "topk10", "topk50", "topk50_topp0.95", "topp0.95"]
BATCHES = [1, 32]


def main(path):
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    calls = []
    for r in rows:
        name = r["Kernel_Name"]
        if not name.startswith(("sample_", "void sample_")):
            continue
        t = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        if "sample_mwg_kernel" in name or not calls:
            calls.append(t)
        else:  # the closing one-workgroup kernel of the call before
            calls[-1] += t
    per = 205
    need = per * len(MODES) * len(BATCHES)
    if len(calls) < need:
        raise SystemExit(f"expected {need} sampler calls, found {len(calls)}")
    calls = calls[-need:]
    print("| batch | mode | kernel us per call (median of 200) |")
    print("|---|---|---|")
    i = 0
    for b in BATCHES:
        for m in MODES:
            seg = calls[i + 5:i + per]
            print(f"| {b} | {m} | {statistics.median(seg):.1f} |")
            i += per


if __name__ == "__main__":
    main(sys.argv[1])
