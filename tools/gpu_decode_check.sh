#!/bin/bash
# MI355X decode-path check: decode kernel/engine tests, GPT-J decode-only ms/step at B=1/8/32
# (contiguous and paged KV), the full decode_bench table, and a rocprofv3 kernel trace of the B=1 step.
set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_decode_gpu.py > gpurun_out/dec_tests.log 2>&1 || exit 1
for B in 1 8 32; do
  timeout -k 10 200 python -u bench/decode_bench.py --batches $B --decode-only 40 --page-size 0 > gpurun_out/dec_b${B}_contig.log 2>&1 && \
  timeout -k 10 200 python -u bench/decode_bench.py --batches $B --decode-only 40 > gpurun_out/dec_b${B}_paged.log 2>&1 || exit 1
done
timeout -k 10 400 python -u bench/decode_bench.py > gpurun_out/decode_full.log 2>&1 && \
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/dec_prof -o dec -- python3 $GRAFT_REPO_ROOT/bench/decode_bench.py --batches 1 --decode-only 40 > $GRAFT_REPO_ROOT/gpurun_out/dec_prof.log 2>&1
