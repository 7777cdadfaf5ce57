#!/bin/bash
# batched small-gradient accumulation: tests (kernel, ZeRO world-2 on GPU), DreamBooth A/B, profile
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_unet_fusions_gpu.py -k "accum or phase or training" -x -q --timeout 200 --timeout-method thread > gpurun_out/acc_k.log 2>&1 || { tail -20 gpurun_out/acc_k.log; exit 1; }
tail -1 gpurun_out/acc_k.log
GPU_AB_TESTS="tests/test_multirank_gpu.py tests/test_entrypoints_gpu.py" bash tools/gpu_ab.sh acc 2 \
  "KCA_MULTI_ACCUM=0 KCA_SD_PHASE_UP_TRAIN=0" "KCA_MULTI_ACCUM=1 KCA_SD_PHASE_UP_TRAIN=1" 300 python -u bench/sd_bench.py --mode train --steps 8 --warmup 3 || exit 1
cd /tmp && timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/sdt_prof2 -o sdt -- python3 $GRAFT_REPO_ROOT/bench/sd_bench.py --mode train --steps 4 --warmup 2 > $GRAFT_REPO_ROOT/gpurun_out/sdt_prof2.log 2>&1 || exit 4
echo profiled
