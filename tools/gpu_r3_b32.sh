#!/bin/bash
# batch-32 decode: GELU route (eager chain / native in-place / hipBLASLt epilogue) and split-K target
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
CMD="python -u bench/decode_bench.py --batches 32 --decode-only 24"
GPU_AB_TESTS="tests/test_decode_gpu.py" bash tools/gpu_ab.sh b32gelu 2 "KCA_DECODE_GELU=torch" "KCA_DECODE_GELU=native" 300 $CMD &&
bash tools/gpu_ab.sh b32epi 1 "KCA_DECODE_GELU=native" "KCA_DECODE_GELU=epi" 300 $CMD &&
bash tools/gpu_ab.sh b32wgs 1 "KCA_DECODE_WGS=256" "KCA_DECODE_WGS=1024" 300 $CMD &&
bash tools/gpu_ab.sh b32wgs2 1 "KCA_DECODE_WGS=256" "KCA_DECODE_WGS=2048" 300 $CMD
