# round-4 batch 3: sampler segment stamps, multi-rank training rehearsals, SD batch
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
KCA_KERNEL_LIB=$PWD/ab/libkca_kernels_stamps.so timeout -k 10 120 python -u tools/sample_stamps.py --modes greedy,topk10,topk50,topk50_topp0.95 > gpurun_out/sampler_stamps_r4.txt 2>&1 || { tail -20 gpurun_out/sampler_stamps_r4.txt; exit 1; }
cat gpurun_out/sampler_stamps_r4.txt
timeout -k 10 800 python -u -m pytest tests/test_multirank_train_gpu.py -x -v --timeout 400 --timeout-method thread > gpurun_out/multirank_r4.log 2>&1; rc=$?
tail -12 gpurun_out/multirank_r4.log
[ $rc -eq 0 ] || exit $rc
bash tools/gpu_r4_sd.sh
