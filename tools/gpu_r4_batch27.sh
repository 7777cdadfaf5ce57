# round-4 batch 27: B=1 attention splits in one pass of 8 tokens per lane group (KCA_DEC_U8) -- A/B + stamps
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
KCA_DEC_U8=1 timeout -k 10 300 python -u -m pytest tests/test_decode_gpu.py -x -q --timeout 120 --timeout-method thread -k "engine_fused" > gpurun_out/u8_tests.log 2>&1 || { tail -30 gpurun_out/u8_tests.log; exit 1; }
tail -1 gpurun_out/u8_tests.log
for m in 1 0 1 0; do
  KCA_DEC_U8=$m timeout -k 10 240 python -u bench/decode_bench.py --batches 1 --decode-only 200 2>gpurun_out/dec_ab.err | tail -1 | cut -c1-100 || { tail -20 gpurun_out/dec_ab.err; exit 1; }
  echo "  (u8=$m)"
done
timeout -k 10 300 python -u bench/decode_layer_stamps.py --steps 8 2> gpurun_out/dec_stamps.err | tee gpurun_out/dec_layer_stamps_desc_r4.jsonl || { tail -20 gpurun_out/dec_stamps.err; exit 1; }
