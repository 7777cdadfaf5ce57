#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_attention_masks_gpu.py tests/test_kernels_gpu.py tests/test_decode_gpu.py \
  -v --timeout 200 --timeout-method thread > gpurun_out/r3_masks.log 2>&1
echo "rc=$?"; tail -4 gpurun_out/r3_masks.log
