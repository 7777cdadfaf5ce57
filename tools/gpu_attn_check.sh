#!/bin/bash
# Attention kernels on MI355X: numerics tests, micro-benchmark, and a per-kernel trace of the bench.
set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
SHAPES=${SHAPES:-gptj,gpt2,bloom_tp8,sd_64,sd_32}
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_kernels_gpu.py -k "attention or attn or sd_fused" > gpurun_out/attn_tests.log 2>&1 && \
timeout -k 10 300 python -u bench/attn_bench.py --shapes $SHAPES --no-sdpa > gpurun_out/attn_bench.log 2>&1 && \
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/attn_prof -o attn -- python3 $GRAFT_REPO_ROOT/bench/attn_bench.py --shapes gptj --no-sdpa > $GRAFT_REPO_ROOT/gpurun_out/attn_prof.log 2>&1
