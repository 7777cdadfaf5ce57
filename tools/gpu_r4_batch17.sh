# round-4 batch 17: two-bias residual add (UNet training) tests + DreamBooth, then the GPT-J TunableOp re-tune A/B
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_unet_fusions_gpu.py tests/test_kernels_gpu.py -q --timeout 300 --timeout-method thread > gpurun_out/sd_tests_r4.log 2>&1 || { tail -30 gpurun_out/sd_tests_r4.log; exit 1; }
tail -2 gpurun_out/sd_tests_r4.log
for i in 1 2; do timeout -k 10 300 python -u bench/sd_bench.py --mode train --steps 10 --warmup 3 2>/dev/null | tail -1 | cut -c1-120; done
bash tools/gpu_r4_tune_gptj.sh
