# round-4 batch 28: merged QKV + attention + fc_in launch again, now with the step descriptors
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
for m in 1 0 1 0; do
  KCA_DECODE_MERGED=$m timeout -k 10 240 python -u bench/decode_bench.py --batches 1 --decode-only 200 2>gpurun_out/dec_ab.err | tail -1 | cut -c1-100 || { tail -20 gpurun_out/dec_ab.err; exit 1; }
  echo "  (merged=$m)"
done
