# round-4 batch 8: sampler (single-wave selects) tests + stamps + kernel times, DreamBooth attribution + kernel split
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_decode_gpu.py -q --timeout 200 --timeout-method thread > gpurun_out/decode_tests_r4f.log 2>&1 || { tail -30 gpurun_out/decode_tests_r4f.log; exit 1; }
tail -2 gpurun_out/decode_tests_r4f.log
KCA_KERNEL_LIB=$PWD/ab/libkca_kernels_stamps.so timeout -k 10 120 python -u tools/sample_stamps.py --modes topk10,topk50,topk50_topp0.95 > gpurun_out/sampler_stamps_r4f.txt 2>&1 || { tail -20 gpurun_out/sampler_stamps_r4f.txt; exit 1; }
cat gpurun_out/sampler_stamps_r4f.txt
(cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/sampler_mwg1f -o s --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/sample_bench.py > $GRAFT_REPO_ROOT/gpurun_out/sampler_mwg1f.txt 2>&1) || { echo "sampler prof failed"; exit 1; }
grep "us/call" gpurun_out/sampler_mwg1f.txt
timeout -k 10 300 python -u bench/sd_bench.py --mode train --steps 3 --warmup 2 --attrib > gpurun_out/sdt_attrib_r4c.json 2> gpurun_out/sdt_attrib_r4c.err || { tail -20 gpurun_out/sdt_attrib_r4c.err; exit 1; }
grep -A42 "attrib\]" gpurun_out/sdt_attrib_r4c.err | head -45
(cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/sdt_prof_r4b -o sdt -- python3 $GRAFT_REPO_ROOT/bench/sd_bench.py --mode train --steps 4 --warmup 2 > $GRAFT_REPO_ROOT/gpurun_out/sdt_prof_r4b.log 2>&1) || { echo "train prof failed"; exit 1; }
tail -1 gpurun_out/sdt_prof_r4b.log
