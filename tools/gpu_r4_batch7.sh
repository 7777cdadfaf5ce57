# round-4 batch 7: sampler (thread-max local threshold, compacted merge) tests + stamps + kernel times, then batch 6
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_decode_gpu.py -q --timeout 200 --timeout-method thread > gpurun_out/decode_tests_r4e.log 2>&1 || { tail -30 gpurun_out/decode_tests_r4e.log; exit 1; }
tail -2 gpurun_out/decode_tests_r4e.log
KCA_KERNEL_LIB=$PWD/ab/libkca_kernels_stamps.so timeout -k 10 120 python -u tools/sample_stamps.py --modes topk10,topk50,topk50_topp0.95 > gpurun_out/sampler_stamps_r4e.txt 2>&1 || { tail -20 gpurun_out/sampler_stamps_r4e.txt; exit 1; }
cat gpurun_out/sampler_stamps_r4e.txt
(cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/sampler_mwg1e -o s --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/sample_bench.py > $GRAFT_REPO_ROOT/gpurun_out/sampler_mwg1e.txt 2>&1) || { echo "sampler prof failed"; exit 1; }
grep "us/call" gpurun_out/sampler_mwg1e.txt
bash tools/gpu_r4_batch6.sh
