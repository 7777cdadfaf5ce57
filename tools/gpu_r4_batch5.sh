# round-4 batch 5: the whole GPU suite, sampler stamps + kernel times, DreamBooth attribution + bench
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/gpu_suite_r4.log 2>&1 || { tail -40 gpurun_out/gpu_suite_r4.log; exit 1; }
tail -3 gpurun_out/gpu_suite_r4.log
KCA_KERNEL_LIB=$PWD/ab/libkca_kernels_stamps.so timeout -k 10 120 python -u tools/sample_stamps.py --modes topk10,topk50,topk50_topp0.95 > gpurun_out/sampler_stamps_r4d.txt 2>&1 || { tail -20 gpurun_out/sampler_stamps_r4d.txt; exit 1; }
cat gpurun_out/sampler_stamps_r4d.txt
(cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/sampler_mwg1d -o s --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/sample_bench.py > $GRAFT_REPO_ROOT/gpurun_out/sampler_mwg1d.txt 2>&1) || { echo "sampler prof failed"; exit 1; }
grep "us/call" gpurun_out/sampler_mwg1d.txt
timeout -k 10 300 python -u bench/sd_bench.py --mode train --steps 6 --warmup 2 --attrib > gpurun_out/sdt_attrib_r4b.json 2> gpurun_out/sdt_attrib_r4b.err || { tail -20 gpurun_out/sdt_attrib_r4b.err; exit 1; }
grep -A42 "attrib\]" gpurun_out/sdt_attrib_r4b.err | head -45; cat gpurun_out/sdt_attrib_r4b.json
