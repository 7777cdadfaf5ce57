# Attention loop anatomy: in-kernel segment stamps (diagnostic build) for the GPT-J and NeoX shapes.
set -o pipefail
mkdir -p gpurun_out
for s in ${SHAPES:-gptj}; do
  KCA_KERNEL_LIB=$PWD/ab/libkca_kernels_stamps.so timeout -k 10 120 python -u bench/attn_stamps.py --shape $s >> gpurun_out/attn_stamps.jsonl || exit 1
done
cat gpurun_out/attn_stamps.jsonl
