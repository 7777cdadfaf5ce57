#!/bin/bash
# A/B of the M=1 LayerNorm+GEMV split (KCA_DECODE_LN_SPLIT) on GPT-J decode B=1, plus B=8,
# then the decode GPU tests and a kernel trace of the B=1 step.
set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
KCA_DECODE_LN_SPLIT=0 timeout -k 10 200 python -u bench/decode_bench.py --batches 1 --decode-only 40 > gpurun_out/ab_fused.log 2>&1 && \
KCA_DECODE_LN_SPLIT=1 timeout -k 10 200 python -u bench/decode_bench.py --batches 1 --decode-only 40 > gpurun_out/ab_split.log 2>&1 && \
timeout -k 10 200 python -u bench/decode_bench.py --batches 8 --decode-only 40 > gpurun_out/ab_b8.log 2>&1 && \
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_decode_gpu.py > gpurun_out/dec_tests.log 2>&1 && \
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/dec_prof -o dec -- python3 $GRAFT_REPO_ROOT/bench/decode_bench.py --batches 1 --decode-only 40 > $GRAFT_REPO_ROOT/gpurun_out/dec_prof.log 2>&1
