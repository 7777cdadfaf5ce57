#!/bin/bash
# compact top-k sampler: decode tests, decode-only A/B at batch 1 and 32, then a batch-32 timeline
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
GPU_AB_TESTS="tests/test_decode_gpu.py" bash tools/gpu_ab.sh samp1 2 "KCA_SAMPLE_COMPACT=0" "KCA_SAMPLE_COMPACT=1" 300 \
  python -u bench/decode_bench.py --batches 1 --decode-only 48 &&
bash tools/gpu_ab.sh samp32 1 "KCA_SAMPLE_COMPACT=0" "KCA_SAMPLE_COMPACT=1" 300 \
  python -u bench/decode_bench.py --batches 32 --decode-only 24 &&
B=32 bash tools/gpu_decode_timeline.sh && python3 tools/timeline.py gpurun_out/dec_tl/dec_kernel_trace.csv --show 40 > gpurun_out/dec_tl_b32.txt
