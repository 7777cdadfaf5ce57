# LayerNorm backward for narrow rows: tests, then DreamBooth A/B (KCA_LN_BWD_NARROW=0 / 1)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "layernorm or layer_norm" -x -q --timeout 120 --timeout-method thread > gpurun_out/ln_tests.log 2>&1 || { tail -30 gpurun_out/ln_tests.log; exit 1; }
tail -1 gpurun_out/ln_tests.log
: > gpurun_out/ln_ab.log
for rep in 1 2; do
  for S in 0 1; do
    KCA_LN_BWD_NARROW=$S timeout -k 10 300 python -u bench/sd_bench.py --mode train --steps 10 > gpurun_out/ln_${S}_$rep.log 2>&1 || exit 1
    echo "ln_narrow=$S rep=$rep $(grep -h '^{' gpurun_out/ln_${S}_$rep.log | grep -o '"value": [0-9.]*\|"loss": [0-9.]*' | tr '\n' ' ')" | tee -a gpurun_out/ln_ab.log
  done
done
