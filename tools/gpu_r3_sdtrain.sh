#!/bin/bash
# DreamBooth training fusions: parity tests, then an interleaved A/B of the training step
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
GPU_AB_TESTS="tests/test_unet_fusions_gpu.py tests/test_attention_masks_gpu.py" bash tools/gpu_ab.sh sdt 2 \
  "KCA_SD_FOLD_BIAS_TRAIN=0 KCA_SD_FUSED_QKV_TRAIN=0" "KCA_SD_FOLD_BIAS_TRAIN=1" 300 python -u bench/sd_bench.py --mode train --steps 8 --warmup 3
