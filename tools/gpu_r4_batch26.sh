# round-4 batch 26: per-step RoPE / page-row descriptors for the B=1 attention chain -- tests, A/B, stamps
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_decode_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/desc_tests.log 2>&1 || { tail -30 gpurun_out/desc_tests.log; exit 1; }
tail -2 gpurun_out/desc_tests.log
for m in 1 0 1 0; do
  KCA_DECODE_STEP_DESC=$m timeout -k 10 240 python -u bench/decode_bench.py --batches 1 --decode-only 200 2>gpurun_out/dec_ab.err | tail -1 | cut -c1-100 || { tail -20 gpurun_out/dec_ab.err; exit 1; }
  echo "  (step_desc=$m)"
done
