#!/bin/bash
# graph captures in thread-local mode: graph / TP / SD GPU tests, then the driver's default bench twice
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 400 python -u -m pytest tests/test_decode_gpu.py tests/test_tp_engine_gpu.py tests/test_unet_fusions_gpu.py -q -x \
  --timeout 240 --timeout-method thread > gpurun_out/final_tests.log 2>&1 || { tail -30 gpurun_out/final_tests.log; exit 1; }
tail -1 gpurun_out/final_tests.log
for i in 1; do
  timeout -k 10 500 python -u bench.py > gpurun_out/final_bench$i.out 2> gpurun_out/final_bench$i.err || { echo "bench $i rc=$?"; grep -v "^frame" gpurun_out/final_bench$i.err | tail -20; exit 3; }
  grep "^\[bench\]" gpurun_out/final_bench$i.err
done
