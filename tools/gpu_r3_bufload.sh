#!/bin/bash
# Buffer-resource K/V staging in the tiled attention kernels: numerics, then a
# same-box A/B against the flat-address build (ab/libkca_kernels_kca_attn_flat_loads.so)
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_attention_masks_gpu.py -x -q --timeout 200 --timeout-method thread \
  > gpurun_out/r3_buf_tests.log 2>&1 || { tail -30 gpurun_out/r3_buf_tests.log; exit 1; }
tail -2 gpurun_out/r3_buf_tests.log
FLAT=$PWD/ab/libkca_kernels_kca_attn_flat_loads.so
for rep in 1 2; do
  timeout -k 10 300 python -u bench/attn_bench.py --no-sdpa --shapes sd_64_pad64,gpt2,gptj,sd_32_pad96,sd_16 > gpurun_out/r3_attn_buf_${rep}.jsonl 2>&1 || exit 2
  KCA_KERNEL_LIB=$FLAT timeout -k 10 300 python -u bench/attn_bench.py --no-sdpa --shapes sd_64_pad64,gpt2,gptj,sd_32_pad96,sd_16 > gpurun_out/r3_attn_flat_${rep}.jsonl 2>&1 || exit 2
  echo "== rep $rep buf"; cat gpurun_out/r3_attn_buf_${rep}.jsonl; echo "== rep $rep flat"; cat gpurun_out/r3_attn_flat_${rep}.jsonl
done
for rep in 1 2; do
  timeout -k 10 300 python -u bench/sd_bench.py --mode infer --steps 4 > gpurun_out/r3_sd_buf_${rep}.jsonl 2>/dev/null || exit 3
  KCA_KERNEL_LIB=$FLAT timeout -k 10 300 python -u bench/sd_bench.py --mode infer --steps 4 > gpurun_out/r3_sd_flat_${rep}.jsonl 2>/dev/null || exit 3
  echo "sd buf $(cat gpurun_out/r3_sd_buf_${rep}.jsonl)"; echo "sd flat $(cat gpurun_out/r3_sd_flat_${rep}.jsonl)"
done
