#!/usr/bin/env python3
"""Timeline of one step of a rocprofv3 kernel trace: every dispatch of the last complete step
(between two dispatches of --step-kernel) with its start offset, duration, queue and the gap
since the previous dispatch on any queue ended; plus, per kernel name, the time the GPU ran it
with nothing else running ("exposed") -- the part of the step it alone holds.

    python tools/timeline.py gpurun_out/dec_prof/dec_kernel_trace.csv --step-kernel sample_kernel
"""
import argparse
import collections
import csv


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--step-kernel", default="sample_kernel")
    ap.add_argument("--steps", type=int, default=10, help="steps averaged for the exposed-time table")
    ap.add_argument("--show", type=int, default=40, help="dispatches of the last step to list")
    a = ap.parse_args()
    rows = sorted(csv.DictReader(open(a.trace)), key=lambda r: int(r["Start_Timestamp"]))
    marks = [i for i, r in enumerate(rows) if r["Kernel_Name"].startswith(a.step_kernel)]
    lo = marks[-a.steps - 1] + 1
    seg = rows[lo:marks[-1] + 1]
    t0 = int(seg[0]["Start_Timestamp"])
    ev = [(int(r["Start_Timestamp"]) - t0, int(r["End_Timestamp"]) - t0, r["Kernel_Name"].split("(")[0][:48],
           int(r["Grid_Size_X"]) // max(1, int(r["Workgroup_Size_X"])), r.get("Queue_Id", r.get("Stream_Id", "?")))
          for r in seg]
    span = max(e[1] for e in ev)
    # exposed time per name: sweep over elementary intervals
    pts = sorted({p for e in ev for p in (e[0], e[1])})
    exposed = collections.defaultdict(float)
    busy = 0.0
    idle = 0.0
    for x0, x1 in zip(pts, pts[1:]):
        act = [e for e in ev if e[0] <= x0 and e[1] >= x1]
        if not act:
            idle += x1 - x0
            continue
        busy += x1 - x0
        if len(act) == 1:
            exposed[(act[0][2], act[0][3])] += x1 - x0
        else:
            exposed[("(overlapped)", 0)] += x1 - x0
    n = a.steps
    print(f"steps {n}: span/step {span / n / 1e3:.1f} us, busy {busy / n / 1e3:.1f} us, idle {idle / n / 1e3:.1f} us")
    print(f"{'exposed us/step':>16}  kernel (grid)")
    for (k, g), v in sorted(exposed.items(), key=lambda kv: -kv[1]):
        print(f"{v / n / 1e3:16.1f}  {k} ({g})")
    last = [e for e in ev if e[0] >= (int(rows[marks[-2]]["End_Timestamp"]) - t0)]
    print(f"\nlast step, first {a.show} dispatches: start_us dur_us gap_us queue kernel(grid)")
    prev_end = last[0][0]
    for s, e, k, g, q in last[:a.show]:
        print(f"{s / 1e3:9.1f} {(e - s) / 1e3:7.1f} {(s - prev_end) / 1e3:7.1f} {q:>4} {k} ({g})")
        prev_end = max(prev_end, e)


if __name__ == "__main__":
    main()
