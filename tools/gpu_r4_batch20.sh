# round-4 batch 20: B=1 decode layer-kernel A/B -- shipped vs no attention chain in the fc_in kernel vs
# no arrival/LayerNorm tail in the out-projection kernel (timing only; the A/B libraries compute wrong tokens)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
for lib in "" ab/libkca_kernels_kca_ab_no_dec_attn.so ab/libkca_kernels_kca_ab_no_dual_tail.so "" ab/libkca_kernels_kca_ab_no_dec_attn.so ab/libkca_kernels_kca_ab_no_dual_tail.so; do
  KCA_KERNEL_LIB=${lib:+$PWD/$lib} timeout -k 10 240 python -u bench/decode_bench.py --batches 1 --decode-only 200 2>gpurun_out/dec_ab.err | tail -1 || { tail -20 gpurun_out/dec_ab.err; exit 1; }
  echo "  (${lib:-shipped})"
done
