# round-4 batch 25: weight gradients accumulated by the GEMM into the fp32 buffer -- tests + headline A/B
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 200 --timeout-method thread -k "engine or fused or tlinear or block" > gpurun_out/gemm_acc_tests.log 2>&1 || { tail -30 gpurun_out/gemm_acc_tests.log; exit 1; }
tail -2 gpurun_out/gemm_acc_tests.log
for a in 1 0 1 0; do
  KCA_WGRAD_GEMM_ACC=$a timeout -k 10 400 python -u bench.py --steps 5 --warmup 2 --sd 0 --extra off --bloom-tp off 2>gpurun_out/acc_ab.err | tail -1 | cut -c1-140 || { tail -20 gpurun_out/acc_ab.err; exit 1; }
  echo "  (gemm_acc=$a)"
done
