# round-4 batch: sampler tests + kernel times (multi-workgroup vs register kernel), serving bench, multi-rank training rehearsals
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_attention_masks_gpu.py -x -q --timeout 200 --timeout-method thread -k "narrow or unet or wide or vae" > gpurun_out/narrow_tests_r4.log 2>&1 || { tail -30 gpurun_out/narrow_tests_r4.log; exit 1; }
tail -2 gpurun_out/narrow_tests_r4.log
timeout -k 10 300 python -u -m pytest tests/test_decode_gpu.py -x -q --timeout 200 --timeout-method thread -k sample > gpurun_out/sampler_tests_r4.log 2>&1 || { tail -30 gpurun_out/sampler_tests_r4.log; exit 1; }
tail -2 gpurun_out/sampler_tests_r4.log
for arm in 1 0; do
  (cd /tmp && KCA_SAMPLE_MWG=$arm timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/sampler_mwg$arm -o s --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/sample_bench.py > $GRAFT_REPO_ROOT/gpurun_out/sampler_mwg$arm.txt 2>&1) || { echo "sampler arm $arm failed"; exit 1; }
  grep "us/call" gpurun_out/sampler_mwg$arm.txt
done
timeout -k 10 300 python -u bench/serving_bench.py > gpurun_out/serving_r4_v2.jsonl 2>gpurun_out/serving_r4_v2.err || { tail -20 gpurun_out/serving_r4_v2.err; exit 1; }
cat gpurun_out/serving_r4_v2.jsonl
timeout -k 10 700 python -u -m pytest tests/test_multirank_train_gpu.py tests/test_tp_engine_gpu.py -x -v --timeout 400 --timeout-method thread > gpurun_out/multirank_r4.log 2>&1; rc=$?
tail -15 gpurun_out/multirank_r4.log
exit $rc
