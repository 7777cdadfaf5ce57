# round-4 batch 33: K/V prefetch across iterations in the standalone decode attention (batched decode)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_decode_gpu.py tests/test_tp_engine_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/pf_tests.log 2>&1 || { tail -30 gpurun_out/pf_tests.log; exit 1; }
tail -1 gpurun_out/pf_tests.log
for lib in "" ab/libkca_kernels_kca_ab_no_pf.so "" ab/libkca_kernels_kca_ab_no_pf.so; do
  KCA_KERNEL_LIB=${lib:+$PWD/$lib} timeout -k 10 240 python -u bench/decode_bench.py --batches 32 --decode-only 100 2>gpurun_out/dec_ab.err | tail -1 | cut -c1-100 || { tail -20 gpurun_out/dec_ab.err; exit 1; }
  echo "  (B=32 ${lib:-prefetch})"
done
for lib in "" ab/libkca_kernels_kca_ab_no_pf.so; do
  KCA_KERNEL_LIB=${lib:+$PWD/$lib} timeout -k 10 240 python -u bench/decode_bench.py --batches 8 --decode-only 100 2>gpurun_out/dec_ab.err | tail -1 | cut -c1-100 || { tail -20 gpurun_out/dec_ab.err; exit 1; }
  echo "  (B=8 ${lib:-prefetch})"
done
