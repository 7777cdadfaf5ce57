# K-split target sweep of the batched decode GEMM with the packed weight stream (same box)
export TMPDIR=/tmp
mkdir -p gpurun_out/pks
for t in 0 384 768 1024; do
  KCA_MM_TARGET_WG=$t timeout -k 10 300 python bench/decode_suite.py --models gptj,neox --batches 8 > gpurun_out/pks/suite_t$t.jsonl 2>/dev/null || exit 1
  KCA_MM_TARGET_WG=$t timeout -k 10 300 python bench/bloom_tp_bench.py --emulate-tp 8 --batches 8 > gpurun_out/pks/bloom_t$t.jsonl 2>/dev/null || exit 1
  echo "done $t"
done
