#!/bin/bash
# Round-end style MI355X check: the whole GPU test suite, then bench.py (GPT-J headline + SD + BLOOM TP phase).
set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 1500 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_full.log 2>&1; rc=$?
tail -3 gpurun_out/gpu_tests_full.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u bench.py > gpurun_out/bench_full.log 2>&1
