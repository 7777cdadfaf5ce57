#!/bin/bash
# runs on the GPU box: D=64 dK/dV at 3 waves per SIMD (ab build) vs the shipped build, DreamBooth step
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
mkdir -p gpurun_out
OCC3="$PWD/ab/libkca_kernels_kca_ab_dkdv64_occ3.so"
KCA_KERNEL_LIB=$OCC3 timeout -k 10 300 python -u -m pytest tests/test_attention_masks_gpu.py tests/test_kernels_gpu.py -q --timeout 200 --timeout-method thread -k "narrow or tiled or head_dims" -p no:cacheprovider > gpurun_out/occ3_tests.log 2>&1 || { tail -20 gpurun_out/occ3_tests.log; exit 1; }
tail -1 gpurun_out/occ3_tests.log
for lib in default occ3 default occ3; do
  if [ $lib = default ]; then L=""; else L=$OCC3; fi
  KCA_KERNEL_LIB=$L timeout -k 10 240 python -u bench/sd_bench.py --mode train --steps 6 --warmup 2 > gpurun_out/absd_$lib.log 2>&1 || exit 1
  echo "sd_train $lib $(grep -o '"value": [0-9.]*' gpurun_out/absd_$lib.log | head -1) $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/absd_$lib.log | head -1)"
done
