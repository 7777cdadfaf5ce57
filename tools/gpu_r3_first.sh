#!/bin/bash
# Round-3 first GPU pass: custom AR + all-gather, multi-rank rehearsal, bench with N=1 secondaries.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -u -m pytest -x -v --timeout 450 --timeout-method thread \
  tests/test_custom_ar_gpu.py tests/test_multirank_gpu.py > gpurun_out/r3_multirank.log 2>&1
echo "multirank rc=$?"
timeout -k 10 540 python -u bench.py --steps 5 --warmup 2 > gpurun_out/r3_bench1.out 2> gpurun_out/r3_bench1.err
echo "bench rc=$?"
tail -3 gpurun_out/r3_bench1.out
