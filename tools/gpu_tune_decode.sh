#!/bin/bash
# TunableOp search for the serving GEMMs (decode buckets 2..64 + prefill) of GPT-J, then an A/B with the table.
set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
F=gpurun_out/tunableop_decode.csv
rm -f $F
( while true; do date >> gpurun_out/heartbeat.txt; sleep 50; done ) &
HB=$!
KCA_TUNABLEOP=off timeout -k 10 300 python -u bench/decode_bench.py --batches 64 --decode-only 20 > gpurun_out/dt_base64.log 2>&1 && \
KCA_TUNABLEOP=off timeout -k 10 300 python -u bench/decode_bench.py --batches 16 --decode-only 20 > gpurun_out/dt_base16.log 2>&1 && \
timeout -k 10 900 python -u bench/decode_bench.py --no-graphs --batches 2,4,8,16,32,64 --new-tokens 4 --tune $F > gpurun_out/dt_tune.log 2>&1 && \
cp $F tuning/tunableop_decode.csv && \
timeout -k 10 300 python -u bench/decode_bench.py --batches 64 --decode-only 20 > gpurun_out/dt_use64.log 2>&1 && \
timeout -k 10 300 python -u bench/decode_bench.py --batches 16 --decode-only 20 > gpurun_out/dt_use16.log 2>&1
rc=$?
kill $HB
exit $rc
