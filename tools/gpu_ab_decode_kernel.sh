mkdir -p gpurun_out
for B in 1 8 32; do
 for rep in 1 2; do
  KCA_KERNEL_LIB=$PWD/ab/libkca_kernels_old_decode.so timeout -k 10 200 python -u bench/decode_bench.py --batches $B --decode-only 40 > gpurun_out/ab_old_${B}_$rep.log 2>&1 || exit 1
  timeout -k 10 200 python -u bench/decode_bench.py --batches $B --decode-only 40 > gpurun_out/ab_new_${B}_$rep.log 2>&1 || exit 1
 done
done
