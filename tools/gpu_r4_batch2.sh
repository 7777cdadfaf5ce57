# round-4 batch 2: sampler (DPP radix select) tests + kernel times, multi-rank training rehearsals, SD batch
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_decode_gpu.py -x -q --timeout 200 --timeout-method thread -k sample > gpurun_out/sampler_tests_r4b.log 2>&1 || { tail -30 gpurun_out/sampler_tests_r4b.log; exit 1; }
tail -2 gpurun_out/sampler_tests_r4b.log
(cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/sampler_mwg1b -o s --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/sample_bench.py > $GRAFT_REPO_ROOT/gpurun_out/sampler_mwg1b.txt 2>&1) || { echo "sampler prof failed"; exit 1; }
grep "us/call" gpurun_out/sampler_mwg1b.txt
timeout -k 10 800 python -u -m pytest tests/test_multirank_train_gpu.py -x -v --timeout 400 --timeout-method thread > gpurun_out/multirank_r4.log 2>&1; rc=$?
tail -12 gpurun_out/multirank_r4.log
[ $rc -eq 0 ] || exit $rc
bash tools/gpu_r4_sd.sh
