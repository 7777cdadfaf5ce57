#!/bin/bash
# runs on the GPU box (temporary A/B driver, round 5)
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_decode_gpu.py -q --timeout 200 --timeout-method thread -k "dual_ln or layer_kinds or emulated or bit_identical" -p no:cacheprovider > gpurun_out/t9.log 2>&1 || { tail -20 gpurun_out/t9.log; exit 1; }
tail -1 gpurun_out/t9.log
R2="$PWD/ab/libkca_kernels_kca_ab_gemv_r2.so"
for lib in default r2 default r2; do
  if [ $lib = default ]; then L=""; else L=$R2; fi
  KCA_KERNEL_LIB=$L timeout -k 10 240 python -u bench/bloom_tp_bench.py --emulate-tp 8 --batches 1 --new-tokens 64 > gpurun_out/ab5_bloom_$lib.log 2>&1 || exit 1
  echo "bloom $lib $(grep -o '"decode_ms_per_token": [0-9.]*' gpurun_out/ab5_bloom_$lib.log)"
  KCA_KERNEL_LIB=$L timeout -k 10 200 python -u bench/decode_bench.py --batches 1 --new-tokens 64 > gpurun_out/ab5_gptj_$lib.log 2>&1 || exit 1
  echo "gptj $lib $(grep -o '"decode_ms_per_step": [0-9.]*' gpurun_out/ab5_gptj_$lib.log)"
done
bash tools/ab_sd_dkdv.sh
