# round-4 batch 32: GEMM-side gradient accumulation actually engaged (fp32 accumulator guard fixed) -- test + A/B
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 200 --timeout-method thread -k "engine or fused or block" > gpurun_out/gemm_acc_tests2.log 2>&1 || { tail -30 gpurun_out/gemm_acc_tests2.log; exit 1; }
tail -1 gpurun_out/gemm_acc_tests2.log
for a in 1 0 1 0; do
  KCA_WGRAD_GEMM_ACC=$a timeout -k 10 400 python -u bench.py --steps 5 --warmup 2 --sd 0 --extra off --bloom-tp off 2>gpurun_out/acc_ab.err | tail -1 | cut -c1-140 || { tail -20 gpurun_out/acc_ab.err; exit 1; }
  echo "  (gemm_acc=$a)"
done
