# GPT-J decode A/B on one box: the committed kernel library + the earlier split policy
# (ab/libkca_kernels_head.so, KCA_DECODE_SPLIT_POLICY=wgs1024) against the working tree.
mkdir -p gpurun_out
for B in ${BATCHES:-1 8 32}; do
  KCA_KERNEL_LIB=$PWD/ab/libkca_kernels_head.so KCA_DECODE_SPLIT_POLICY=wgs1024 timeout -k 10 200 python -u bench/decode_bench.py --batches $B --decode-only 40 > gpurun_out/ab2_old_$B.log 2>&1 || exit 1
  timeout -k 10 200 python -u bench/decode_bench.py --batches $B --decode-only 40 > gpurun_out/ab2_new_$B.log 2>&1 || exit 1
  grep -h '^{' gpurun_out/ab2_old_$B.log gpurun_out/ab2_new_$B.log | cut -c1-220
done
