# round-4 batch 22: merged QKV + attention + fc_in decode launch -- tests, same-box A/B, stamps
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_decode_gpu.py -x -q --timeout 120 --timeout-method thread -k "merged or fused or dual" > gpurun_out/merged_tests.log 2>&1 || { tail -30 gpurun_out/merged_tests.log; exit 1; }
tail -2 gpurun_out/merged_tests.log
for m in 1 0 1 0; do
  KCA_DECODE_MERGED=$m timeout -k 10 240 python -u bench/decode_bench.py --batches 1 --decode-only 200 2>gpurun_out/dec_ab.err | tail -1 || { tail -20 gpurun_out/dec_ab.err; exit 1; }
  echo "  (merged=$m)"
done
timeout -k 10 300 python -u bench/decode_layer_stamps.py --steps 8 2> gpurun_out/dec_stamps.err | tee gpurun_out/dec_layer_stamps_merged_r4.jsonl || { tail -20 gpurun_out/dec_stamps.err; exit 1; }
