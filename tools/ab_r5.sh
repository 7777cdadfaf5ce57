#!/bin/bash
# runs on the GPU box (temporary A/B driver, round 5)
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_decode_gpu.py tests/test_attention_masks_gpu.py tests/test_kernels_gpu.py -q --timeout 200 --timeout-method thread -k "dual_ln or layer_kinds or emulated or bit_identical or skinny or gemv or narrow or tiled or head_dims" -p no:cacheprovider > gpurun_out/t10.log 2>&1 || { tail -20 gpurun_out/t10.log; exit 1; }
tail -1 gpurun_out/t10.log
DQ="$PWD/ab/libkca_kernels_kca_ab_dq64_occ4.so"
KCA_KERNEL_LIB=$DQ timeout -k 10 300 python -u -m pytest tests/test_attention_masks_gpu.py tests/test_kernels_gpu.py -q --timeout 200 --timeout-method thread -k "narrow or tiled or head_dims" -p no:cacheprovider > gpurun_out/t11.log 2>&1 || { tail -20 gpurun_out/t11.log; exit 1; }
tail -1 gpurun_out/t11.log
U2="$PWD/ab/libkca_kernels_kca_ab_gemv_u2.so"
for lib in default u2 default u2; do
  if [ $lib = default ]; then L=""; else L=$U2; fi
  KCA_KERNEL_LIB=$L timeout -k 10 240 python -u bench/bloom_tp_bench.py --emulate-tp 8 --batches 1 --new-tokens 64 > gpurun_out/ab6_bloom_$lib.log 2>&1 || exit 1
  echo "bloom $lib $(grep -o '"decode_ms_per_token": [0-9.]*' gpurun_out/ab6_bloom_$lib.log)"
  KCA_KERNEL_LIB=$L timeout -k 10 200 python -u bench/decode_bench.py --batches 1 --new-tokens 64 > gpurun_out/ab6_gptj_$lib.log 2>&1 || exit 1
  echo "gptj $lib $(grep -o '"decode_ms_per_step": [0-9.]*' gpurun_out/ab6_gptj_$lib.log)"
done
for lib in default dq4 default dq4; do
  if [ $lib = default ]; then L=""; else L=$DQ; fi
  KCA_KERNEL_LIB=$L timeout -k 10 240 python -u bench/sd_bench.py --mode train --steps 6 --warmup 2 > gpurun_out/ab6_sd_$lib.log 2>&1 || exit 1
  echo "sd_train $lib $(grep -o '"value": [0-9.]*' gpurun_out/ab6_sd_$lib.log | head -1) $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/ab6_sd_$lib.log | head -1)"
done
