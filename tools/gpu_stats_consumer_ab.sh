# consumer-merged row statistics (KCA_MM_STATS_CONSUMER): GPU tests with the flag on, then a same-box A/B
export TMPDIR=/tmp
mkdir -p gpurun_out/sc
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_skinny_mfma_gpu.py -m gpu -k "consumer or residual or two_jobs" > gpurun_out/sc/t0.log 2>&1 || { tail -30 gpurun_out/sc/t0.log; exit 1; }
tail -1 gpurun_out/sc/t0.log
KCA_MM_STATS_CONSUMER=1 timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_decode_gpu.py tests/test_tp_engine_gpu.py tests/test_custom_ar_gpu.py -m gpu -k "batched or fp16 or tp or fused" > gpurun_out/sc/t1.log 2>&1 || { tail -30 gpurun_out/sc/t1.log; exit 1; }
tail -1 gpurun_out/sc/t1.log
for c in 0 1 0 1; do
  KCA_MM_STATS_CONSUMER=$c timeout -k 10 300 python bench/decode_suite.py --models gptj,neox --batches 8 >> gpurun_out/sc/suite_c$c.jsonl 2>/dev/null || exit 1
  KCA_MM_STATS_CONSUMER=$c timeout -k 10 300 python bench/bloom_tp_bench.py --emulate-tp 8 --batches 8 >> gpurun_out/sc/bloom_c$c.jsonl 2>/dev/null || exit 1
  echo "done $c"
done
