# round-4 batch 30: step descriptors for batched decode + TP; flat arrival A/B for the out-proj kernel
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_decode_gpu.py tests/test_tp_engine_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/desc2_tests.log 2>&1 || { tail -30 gpurun_out/desc2_tests.log; exit 1; }
tail -1 gpurun_out/desc2_tests.log
for m in 1 0 1 0; do
  KCA_DECODE_STEP_DESC=$m timeout -k 10 240 python -u bench/decode_bench.py --batches 32 --decode-only 100 2>gpurun_out/dec_ab.err | tail -1 | cut -c1-100 || { tail -20 gpurun_out/dec_ab.err; exit 1; }
  echo "  (B=32 step_desc=$m)"
done
for m in 1 0 1 0; do
  KCA_DUAL_FLAT=$m timeout -k 10 240 python -u bench/decode_bench.py --batches 1 --decode-only 200 2>gpurun_out/dec_ab.err | tail -1 | cut -c1-100 || { tail -20 gpurun_out/dec_ab.err; exit 1; }
  echo "  (B=1 dual_flat=$m)"
done
