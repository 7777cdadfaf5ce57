#!/bin/bash
# decode lookahead: tests, bench, B=1 timeline
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_decode_gpu.py tests/test_entrypoints_gpu.py tests/test_tp_engine_gpu.py \
  tests/test_attention_masks_gpu.py -x -v --timeout 200 --timeout-method thread > gpurun_out/r3_dec_tests.log 2>&1 || { echo tests failed; tail -30 gpurun_out/r3_dec_tests.log; exit 1; }
tail -2 gpurun_out/r3_dec_tests.log
timeout -k 10 300 python -u bench/decode_bench.py --batches 1,8,32 --prompt-len 512 --new-tokens 64 > gpurun_out/r3_dec_bench.jsonl 2> gpurun_out/r3_dec_bench.err || exit 2
timeout -k 10 200 python -u bench/decode_bench.py --batches 1 --decode-only 100 >> gpurun_out/r3_dec_bench.jsonl 2>> gpurun_out/r3_dec_bench.err || exit 3
timeout -k 10 200 python -u bench/decode_bench.py --batches 32 --decode-only 100 >> gpurun_out/r3_dec_bench.jsonl 2>> gpurun_out/r3_dec_bench.err || exit 4
cat gpurun_out/r3_dec_bench.jsonl
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/dec_tl3 -o dec -- python3 $GRAFT_REPO_ROOT/bench/decode_bench.py --batches 1 --decode-only 40 > $GRAFT_REPO_ROOT/gpurun_out/dec_tl3.log 2>&1 || exit 5
echo done
