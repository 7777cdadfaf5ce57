set -o pipefail
timeout -k 10 300 python -u -m pytest tests/test_skinny_mfma_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/mfma_tests.log 2>&1 || exit 1
for cfg in ${MM_SWEEP_CFGS:-"256 4 1" "256 8 1" "128 8 1" "128 4 1" "128 8 2"}; do
  set -- $cfg
  KCA_MM_KC=$1 KCA_MM_WV=$2 timeout -k 10 120 python -u bench/mm_bench.py --variants mfma --nr $3 --ms 1,8,16,32,64 > gpurun_out/sweep_kc$1_wv$2_nr$3.jsonl 2>/dev/null || exit 2
done
