#!/bin/bash
# Re-tune hipBLASLt/rocBLAS solutions (TunableOp) for the default GPT-J micro-batch and A/B it.
# A heartbeat file keeps the run visibly alive while TunableOp searches a shape silently.
set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
F=gpurun_out/tunableop_gptj_mb16.csv
rm -f $F
( while true; do date >> gpurun_out/heartbeat.txt; sleep 50; done ) &
HB=$!
timeout -k 10 1000 python -u bench.py --steps 2 --warmup 2 --sd 0 --tunableop tune --tunableop-file $F > gpurun_out/tune_run.log 2>&1 && \
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --sd 0 --tunableop use --tunableop-file $F > gpurun_out/tune_use.log 2>&1 && \
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --sd 0 > gpurun_out/tune_base.log 2>&1
rc=$?
kill $HB
exit $rc
