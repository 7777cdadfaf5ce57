# SD: folded conv biases -- kernel + block tests, then txt2img A/B (KCA_SD_FOLD_BIAS=0 / 1), interleaved
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "add_bias or folded or unet or groupnorm" -x -q --timeout 120 --timeout-method thread > gpurun_out/fold_tests.log 2>&1 || { tail -30 gpurun_out/fold_tests.log; exit 1; }
tail -1 gpurun_out/fold_tests.log
: > gpurun_out/fold_ab.log
for rep in 1 2; do
  for F in 0 1; do
    KCA_SD_FOLD_BIAS=$F timeout -k 10 300 python -u bench/sd_bench.py --mode infer --steps 2 > gpurun_out/fold_${F}_$rep.log 2>&1 || exit 1
    echo "fold=$F rep=$rep $(grep -h '^{' gpurun_out/fold_${F}_$rep.log | grep -o '"value": [0-9.]*\|"ms_per_batch": [0-9.]*' | tr '\n' ' ')" | tee -a gpurun_out/fold_ab.log
  done
done
