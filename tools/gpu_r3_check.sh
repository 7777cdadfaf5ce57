#!/bin/bash
# full GPU suite + smoke + the driver's default N=1 bench
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 240 --timeout-method thread > gpurun_out/r3_gpu_tests.log 2>&1
rc=$?
echo "tests rc=$rc"; tail -3 gpurun_out/r3_gpu_tests.log
[ $rc -eq 0 ] || { grep -E "FAILED|Error" gpurun_out/r3_gpu_tests.log | head -20; exit 1; }
timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r3_smoke.log 2>&1 || { tail -20 gpurun_out/r3_smoke.log; exit 2; }
tail -1 gpurun_out/r3_smoke.log
timeout -k 10 900 python -u bench.py > gpurun_out/r3_bench2.out 2> gpurun_out/r3_bench2.err || { echo "bench rc=$?"; tail -20 gpurun_out/r3_bench2.err; exit 3; }
tail -c 2500 gpurun_out/r3_bench2.out
