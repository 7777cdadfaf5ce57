export TMPDIR=/tmp
mkdir -p gpurun_out/pk
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_skinny_mfma_gpu.py tests/test_decode_gpu.py -m gpu -k "packed or batched or mfma" > gpurun_out/pk/tests.log 2>&1 || { tail -30 gpurun_out/pk/tests.log; exit 1; }
tail -1 gpurun_out/pk/tests.log
export KCA_DECODE_BATCHED_MAX_B=64
for v in "0 0" "1 0" "1 128"; do
  set -- $v
  KCA_MM_PACK=$1 KCA_MM_KC=$2 timeout -k 10 300 python bench/decode_suite.py --models gptj,neox --batches 8,32 > gpurun_out/pk/suite_p$1_kc$2.jsonl 2>/dev/null || exit 1
  KCA_MM_PACK=$1 KCA_MM_KC=$2 timeout -k 10 300 python bench/bloom_tp_bench.py --emulate-tp 8 --batches 8,32 > gpurun_out/pk/bloom_p$1_kc$2.jsonl 2>/dev/null || exit 1
  echo "done $v"
done
