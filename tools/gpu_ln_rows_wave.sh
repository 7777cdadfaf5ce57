# Decode LN rows: one wave per row (KCA_LN_ROWS_WAVE=1) vs the 256-thread block kernel (0); tests first
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_decode_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/lnw_tests.log 2>&1 || { tail -30 gpurun_out/lnw_tests.log; exit 1; }
tail -1 gpurun_out/lnw_tests.log
: > gpurun_out/lnw_ab.log
for rep in 1 2 3; do
  for S in 0 1; do
    KCA_LN_ROWS_WAVE=$S timeout -k 10 200 python -u bench/decode_bench.py --batches 1 --decode-only 40 > gpurun_out/lnw_${S}_$rep.log 2>&1 || exit 1
    echo "ln_wave=$S rep=$rep $(grep -h '^{' gpurun_out/lnw_${S}_$rep.log | grep -o '"decode_ms_per_step": [0-9.]*')" | tee -a gpurun_out/lnw_ab.log
  done
done
