#!/bin/bash
# A/B of the side-stream MLP branch (KCA_DECODE_PAR_MLP) on GPT-J decode B=1/8/32, engine tests first.
set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_decode_gpu.py -k "engine or layer_split" > gpurun_out/par_tests.log 2>&1 && \
for B in 1 8 32; do
  KCA_DECODE_PAR_MLP=0 timeout -k 10 200 python -u bench/decode_bench.py --batches $B --decode-only 40 > gpurun_out/par0_b$B.log 2>&1 && \
  KCA_DECODE_PAR_MLP=1 timeout -k 10 200 python -u bench/decode_bench.py --batches $B --decode-only 40 > gpurun_out/par1_b$B.log 2>&1 || exit 1
done && \
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/par_prof -o dec -- python3 $GRAFT_REPO_ROOT/bench/decode_bench.py --batches 1 --decode-only 40 > $GRAFT_REPO_ROOT/gpurun_out/par_prof.log 2>&1
