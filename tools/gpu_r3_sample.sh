#!/bin/bash
# register sampler with 4-bit digit radix selects: decode tests, kernel times per mode, generate A/B
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_decode_gpu.py -q -x --timeout 200 --timeout-method thread \
  > gpurun_out/samp_tests.log 2>&1 || { tail -30 gpurun_out/samp_tests.log; exit 1; }
tail -1 gpurun_out/samp_tests.log
(cd /tmp && timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/samp_prof -o samp -- python3 $GRAFT_REPO_ROOT/tools/sample_bench.py > $GRAFT_REPO_ROOT/gpurun_out/samp_prof.log 2>&1) &&
python3 - <<'PY' &&
import csv, glob, os
f = glob.glob(os.environ["GRAFT_REPO_ROOT"] + "/gpurun_out/samp_prof/**/*kernel_trace.csv", recursive=True)[0]
rows = [r for r in csv.DictReader(open(f)) if "sample" in r["Kernel_Name"]]
n = 205
for mi, name in enumerate(["greedy", "multinomial", "topk50", "topp0.95", "topk50_topp0.95"]):
    seg = rows[mi * n + 5:(mi + 1) * n]
    d = sorted(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in seg)
    print(name, rows[mi * n]["Kernel_Name"][:40], "median us", d[len(d) // 2] / 1000)
PY
bash tools/gpu_ab.sh sampreg_gen 2 "KCA_SAMPLE_REG=0" "KCA_SAMPLE_REG=1" 300 python -u bench/decode_bench.py --batches 1,32 --new-tokens 64
