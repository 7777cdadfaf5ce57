# round-4 batch 29: out-projection kernel arrival -- one flat counter vs 64 sub-counters
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
KCA_DUAL_FLAT=1 timeout -k 10 300 python -u -m pytest tests/test_decode_gpu.py -x -q --timeout 120 --timeout-method thread -k "dual or engine_fused" > gpurun_out/flat_tests.log 2>&1 || { tail -30 gpurun_out/flat_tests.log; exit 1; }
tail -1 gpurun_out/flat_tests.log
for m in 1 0 1 0; do
  KCA_DUAL_FLAT=$m timeout -k 10 240 python -u bench/decode_bench.py --batches 1 --decode-only 200 2>gpurun_out/dec_ab.err | tail -1 | cut -c1-100 || { tail -20 gpurun_out/dec_ab.err; exit 1; }
  echo "  (flat=$m)"
done
