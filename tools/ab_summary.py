#!/usr/bin/env python3
"""Summarise an interleaved A/B log (JSON lines tagged with "lib"): per shape and lib,
the best of the repeats for every numeric *_ms field."""
import json
import sys
from collections import defaultdict

rows = [json.loads(l) for l in open(sys.argv[1]) if l.startswith("{")]
best = defaultdict(dict)
for r in rows:
    k = (r.get("shape"), r["lib"])
    for f, v in r.items():
        if f.endswith("_ms") and isinstance(v, (int, float)):
            best[k][f] = min(best[k].get(f, 1e30), v)
shapes = sorted({k[0] for k in best})
libs = sorted({k[1] for k in best})
for s in shapes:
    for f in sorted(best[(s, libs[0])]):
        vals = [best[(s, l)].get(f) for l in libs]
        print(f"{s:14s} {f:22s} " + "  ".join(f"{l}={v:.3f}" for l, v in zip(libs, vals))
              + (f"  ratio={vals[-1] / vals[0]:.3f}" if len(vals) == 2 else ""))
