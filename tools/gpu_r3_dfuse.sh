#!/bin/bash
# fused batch-1 decode layer: decode tests, then decode-only A/B (two-stream vs fused)
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
bash tools/gpu_ab.sh dfuse 2 "KCA_DUAL_CHUNK=0" "KCA_DUAL_CHUNK=1" 300 \
  python -u bench/decode_bench.py --batches 1 --decode-only 48
