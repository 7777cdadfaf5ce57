# round-4 batch 10: sampler (per-wave narrowing) tests + stamps + kernel times + decode rows
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_decode_gpu.py -q --timeout 200 --timeout-method thread > gpurun_out/decode_tests_r4h.log 2>&1 || { tail -30 gpurun_out/decode_tests_r4h.log; exit 1; }
tail -2 gpurun_out/decode_tests_r4h.log
KCA_KERNEL_LIB=$PWD/ab/libkca_kernels_stamps.so timeout -k 10 120 python -u tools/sample_stamps.py --modes topk10,topk50,topk50_topp0.95 > gpurun_out/sampler_stamps_r4h.txt 2>&1 || { tail -20 gpurun_out/sampler_stamps_r4h.txt; exit 1; }
cat gpurun_out/sampler_stamps_r4h.txt
(cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/sampler_mwg1h -o s --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/sample_bench.py > $GRAFT_REPO_ROOT/gpurun_out/sampler_mwg1h.txt 2>&1) || { echo "sampler prof failed"; exit 1; }
grep "us/call" gpurun_out/sampler_mwg1h.txt
timeout -k 10 300 python -u -c "
import json, sys; sys.path.insert(0, 'bench')
import decode_bench
for r in decode_bench.run_decode('gpt-j-6b', batches=(1, 32), prompt_len=512, new_tokens=64, sampling=('greedy', 'ft_topk10')):
    print(json.dumps(r), flush=True)
" > gpurun_out/decode_r4h.jsonl 2> gpurun_out/decode_r4h.err || { tail -20 gpurun_out/decode_r4h.err; exit 1; }
cat gpurun_out/decode_r4h.jsonl
