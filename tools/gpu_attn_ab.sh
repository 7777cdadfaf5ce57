# Attention A/B on one box: committed kernel library vs working tree, interleaved repeats.
mkdir -p gpurun_out
: > gpurun_out/attn_ab.log
for rep in 1 2; do
  KCA_KERNEL_LIB=$PWD/ab/libkca_kernels_head.so timeout -k 10 200 python -u bench/attn_bench.py --no-sdpa --shapes ${SHAPES:-gptj} | sed 's/^{/{"lib": "head", /' >> gpurun_out/attn_ab.log || exit 1
  timeout -k 10 200 python -u bench/attn_bench.py --no-sdpa --shapes ${SHAPES:-gptj} | sed 's/^{/{"lib": "new", /' >> gpurun_out/attn_ab.log || exit 1
done
grep '^{' gpurun_out/attn_ab.log
