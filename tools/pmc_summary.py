#!/usr/bin/env python3
"""Join the rocprofv3 passes of ``tools/pmc_profile.sh`` into one per-kernel
table of derived gfx950 metrics.

Per kernel (mean over its dispatches):

* ``us``          wall time per dispatch from the un-instrumented kernel-trace pass
* ``clk_ghz``     effective shader clock, GRBM_GUI_ACTIVE / 8 XCDs / dispatch time (counter pass)
* ``mfma_util``   SQ_VALU_MFMA_BUSY_CYCLES / (1024 SIMDs x GRBM_GUI_ACTIVE / 8): share of
                  all SIMD-cycles the matrix cores were busy (1.0 = 2.5 PF/s bf16 at that clock)
* ``mfma_tflops`` SQ_VALU_MFMA_BUSY_CYCLES x 1024 FLOP (bf16 MFMA rate per busy SIMD-cycle)
                  / trace time: what the matrix cores actually executed
* ``model_tflops`` useful FLOPs of the case (bench/kernel_pmc.py model) / trace time
* ``active`` / ``wait_inst`` / ``wait_any``  shares of SQ_WAVE_CYCLES spent issuing, stalled
                  on issue dependencies, parked on s_waitcnt / barriers
* ``lds_conflict`` SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE (extra cycles per LDS cycle)
* ``rd_gbs`` / ``wr_gbs``  FETCH_SIZE x 2 (gfx950 reports half of a wide streaming read,
                  MI355X_MICROARCH.md §HBM) and WRITE_SIZE, in GB/s of trace time
* ``model_gbs``   modelled compulsory bytes of the case / trace time

Usage: python tools/pmc_summary.py gpurun_out/pmc [--md out.md] [--json out.json]
"""
from __future__ import annotations

import argparse
import csv
import glob
import json
import os
import re
from collections import defaultdict

# kernel-name regex -> (case in bench/kernel_pmc.py, FLOP key or None, byte key or None)
CASE_OF = [
    (r"attn_fwd_tiled_kernel<256", "attn_gptj", "fwd_flops", None),
    (r"attn_fwd_w8_kernel<256", "attn_gptj", "fwd_flops", None),
    (r"attn_bwd_dq_tiled_kernel<256", "attn_gptj", "bwd_flops_dq", None),
    (r"attn_bwd_dkdv_tiled_kernel<256", "attn_gptj", "bwd_flops_dkdv", None),
    (r"attn_fwd_tiled_kernel<64, false, -1, 48", "attn_sd_tiled48", "fwd_flops", None),
    (r"attn_bwd_dq_tiled_kernel<64, false, 48", "attn_sd_tiled48", "bwd_flops_dq", None),
    (r"attn_bwd_dkdv_tiled_kernel<64, false, 48", "attn_sd_tiled48", "bwd_flops_dkdv", None),
    (r"attn_fwd_kernel<64, false>", "attn_sd64", "fwd_flops", None),
    (r"attn_bwd_dq_kernel<64, false>", "attn_sd64", "bwd_flops_dq", None),
    (r"attn_bwd_dkdv_kernel<64, false>", "attn_sd64", "bwd_flops_dkdv", None),
    (r"ln_fwd_kernel", "layernorm_gptj", None, "fwd_bytes"),
    (r"ln_bwd_kernel", "layernorm_gptj", None, "bwd_bytes"),
    (r"geglu_fwd_kernel", "geglu_sd", None, "fwd_bytes"),
    (r"geglu_bwd_kernel", "geglu_sd", None, "bwd_bytes"),
    (r"ce_fwd_kernel", "xent_gptj", None, "fwd_bytes"),
    (r"ce_bwd_kernel", "xent_gptj", None, "bwd_bytes"),
    (r"^adamw_kernel", "adamw_512m", None, "bytes"),
    (r"skinny_gemm", "gemv_fcin_m1", None, "bytes"),
    (r"decode_attn_kernel", "decode_attn_b32", None, "bytes"),
    (r"nhwc_", "groupnorm_nhwc_sd", None, None),
]
N_SIMD = 1024  # 256 CUs x 4 SIMDs
MFMA_FLOP_PER_BUSY_CYCLE = 1024  # bf16 dense: 2.5 PF / (1024 SIMDs x 2.4 GHz)


def short(name: str) -> str:
    name = re.sub(r"\(anonymous namespace\)::", "", name)
    name = re.sub(r"^void ", "", name)
    return name.split("(")[0][:60]


def load_counters(path):
    """-> {dispatch_id: (kernel, {counter: value}, dur_ns)}"""
    out = {}
    with open(path) as f:
        for r in csv.DictReader(f):
            d = int(r["Dispatch_Id"])
            ent = out.setdefault(d, [r["Kernel_Name"], {}, int(r["End_Timestamp"]) - int(r["Start_Timestamp"])])
            ent[1][r["Counter_Name"]] = ent[1].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    return out


def per_kernel(dispatches):
    acc = defaultdict(lambda: [0, defaultdict(float), 0.0])
    for kern, ctr, dur in dispatches.values():
        a = acc[kern]
        a[0] += 1
        a[2] += dur
        for k, v in ctr.items():
            a[1][k] += v
    return {k: ({c: v / n for c, v in ctr.items()}, dur / n) for k, (n, ctr, dur) in acc.items()}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("root")
    ap.add_argument("--md")
    ap.add_argument("--json")
    args = ap.parse_args()
    cases = json.load(open(os.path.join(args.root, "cases.json")))
    for c in cases.values():  # split the backward FLOPs between the dQ (1 GEMM pair) and dK/dV kernels
        if "bwd_flops" in c:
            c["bwd_flops_dq"] = c["bwd_flops"] * 2 / 5
            c["bwd_flops_dkdv"] = c["bwd_flops"] * 3 / 5
    trace = {}
    for r in csv.DictReader(open(glob.glob(os.path.join(args.root, "trace", "*kernel_stats.csv"))[0])):
        trace[r["Name"]] = float(r["AverageNs"])
    merged = defaultdict(dict)
    clk = {}
    for p in sorted(glob.glob(os.path.join(args.root, "*", "*counter_collection.csv"))):
        for kern, (ctr, dur) in per_kernel(load_counters(p)).items():
            merged[kern].update(ctr)
            if "GRBM_GUI_ACTIVE" in ctr and dur > 0:
                clk.setdefault(kern, []).append(ctr["GRBM_GUI_ACTIVE"] / 8 / dur)
    rows = []
    for kern, ctr in merged.items():
        match = next((m for m in CASE_OF if re.search(m[0], kern)), None)
        if match is None or kern not in trace or match[1] not in cases:
            continue
        _, case, fkey, bkey = match
        ns = trace[kern]
        ghz = sum(clk[kern]) / len(clk[kern]) if kern in clk else float("nan")
        cyc = ctr.get("GRBM_GUI_ACTIVE", 0) / 8
        wave = ctr.get("SQ_WAVE_CYCLES", 0) or float("nan")
        mf = ctr.get("SQ_VALU_MFMA_BUSY_CYCLES", 0.0)
        row = {
            "kernel": short(kern), "case": case, "us": round(ns / 1e3, 1), "clk_ghz": round(ghz, 2),
            "mfma_util": round(mf / (N_SIMD * cyc), 3) if cyc else None,
            "mfma_tflops": round(mf * MFMA_FLOP_PER_BUSY_CYCLE / ns / 1e3, 1),
            "model_tflops": round(cases[case][fkey] / ns / 1e3, 1) if fkey else None,
            "active": round(ctr.get("SQ_ACTIVE_INST_ANY", 0) / wave, 3),
            "wait_inst": round(ctr.get("SQ_WAIT_INST_ANY", 0) / wave, 3),
            "wait_any": round(ctr.get("SQ_WAIT_ANY", 0) / wave, 3),
            "lds_conflict": (round(ctr["SQ_LDS_BANK_CONFLICT"] / ctr["SQ_LDS_IDX_ACTIVE"], 3)
                             if ctr.get("SQ_LDS_IDX_ACTIVE") else None),
            "rd_gbs": round(ctr.get("FETCH_SIZE", 0) * 2 * 1024 / ns, 0),
            "wr_gbs": round(ctr.get("WRITE_SIZE", 0) * 1024 / ns, 0),
            "model_gbs": round(cases[case][bkey] / ns, 0) if bkey else None,
            "valu_per_wave": round(ctr.get("SQ_INSTS_VALU", 0) / max(ctr.get("SQ_WAVES", 1), 1), 0),
            "lds_per_wave": round(ctr.get("SQ_INSTS_LDS", 0) / max(ctr.get("SQ_WAVES", 1), 1), 0),
        }
        rows.append(row)
    rows.sort(key=lambda r: (r["case"], -r["us"]))
    cols = list(rows[0].keys()) if rows else []
    lines = ["| " + " | ".join(cols) + " |", "|" + "---|" * len(cols)]
    for r in rows:
        lines.append("| " + " | ".join("" if r[c] is None else str(r[c]) for c in cols) + " |")
    text = "\n".join(lines)
    print(text)
    if args.md:
        with open(args.md, "w") as f:
            f.write(text + "\n")
    if args.json:
        with open(args.json, "w") as f:
            json.dump(rows, f, indent=1)


if __name__ == "__main__":
    main()
