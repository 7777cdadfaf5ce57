#!/bin/bash
# runs on the GPU box: interleaved A/B of dual-LN geometry builds
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
mkdir -p gpurun_out
for lib in default r16 r8 u2 gemv_r2; do
  if [ $lib = default ]; then L=""; else L="$PWD/ab/libkca_kernels_kca_ab_$( [ $lib = gemv_r2 ] && echo gemv_r2 || echo dual_$lib ).so"; fi
  KCA_KERNEL_LIB=$L timeout -k 10 240 python -u bench/bloom_tp_bench.py --emulate-tp 8 --batches 1 --new-tokens 64 > gpurun_out/abr_bloom_$lib.log 2>&1 || exit 1
  echo "bloom $lib $(grep -o '"decode_ms_per_token": [0-9.]*' gpurun_out/abr_bloom_$lib.log)"
done
for lib in default u2 gemv_r2 default; do
  if [ $lib = default ]; then L=""; else L="$PWD/ab/libkca_kernels_kca_ab_$( [ $lib = gemv_r2 ] && echo gemv_r2 || echo dual_$lib ).so"; fi
  KCA_KERNEL_LIB=$L timeout -k 10 200 python -u bench/decode_bench.py --batches 1 --new-tokens 64 > gpurun_out/abr_gptj_$lib.log 2>&1 || exit 1
  echo "gptj $lib $(grep -o '"decode_ms_per_step": [0-9.]*' gpurun_out/abr_gptj_$lib.log)"
done
