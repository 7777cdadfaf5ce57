# round-4 batch 4: sampler (readlane reductions, early exit, fixed-slot merge) + decode step head (embed+LN kernel,
# chained tokens on the device, one D2H copy): tests, stamps, kernel times, decode bench + B=1 timeline
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_decode_gpu.py tests/test_attention_masks_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/decode_tests_r4c.log 2>&1 || { tail -30 gpurun_out/decode_tests_r4c.log; exit 1; }
tail -2 gpurun_out/decode_tests_r4c.log
KCA_KERNEL_LIB=$PWD/ab/libkca_kernels_stamps.so timeout -k 10 120 python -u tools/sample_stamps.py --modes topk10,topk50_topp0.95 > gpurun_out/sampler_stamps_r4c.txt 2>&1 || { tail -20 gpurun_out/sampler_stamps_r4c.txt; exit 1; }
cat gpurun_out/sampler_stamps_r4c.txt
(cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/sampler_mwg1c -o s --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/sample_bench.py > $GRAFT_REPO_ROOT/gpurun_out/sampler_mwg1c.txt 2>&1) || { echo "sampler prof failed"; exit 1; }
grep "us/call" gpurun_out/sampler_mwg1c.txt
timeout -k 10 300 python -u -c "
import json, sys; sys.path.insert(0, 'bench')
import decode_bench
for r in decode_bench.run_decode('gpt-j-6b', batches=(1, 32), prompt_len=512, new_tokens=64, sampling=('greedy', 'ft_topk10')):
    print(json.dumps(r), flush=True)
" > gpurun_out/decode_r4c.jsonl 2> gpurun_out/decode_r4c.err || { tail -20 gpurun_out/decode_r4c.err; exit 1; }
cat gpurun_out/decode_r4c.jsonl
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/dec_tl_r4 -o dec -- python3 $GRAFT_REPO_ROOT/bench/decode_bench.py --batches 1 --decode-only 40 > $GRAFT_REPO_ROOT/gpurun_out/dec_tl_r4.log 2>&1) || { echo "timeline failed"; tail -5 gpurun_out/dec_tl_r4.log; exit 1; }
tail -2 gpurun_out/dec_tl_r4.log
