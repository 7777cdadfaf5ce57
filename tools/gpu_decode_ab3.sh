# GPT-J decode, split-policy / kernel matrix on one box (bench/decode_bench.py --decode-only).
mkdir -p gpurun_out
run() {  # name, env...
  local name=$1; shift
  for B in ${BATCHES:-1 8}; do
    env "$@" timeout -k 10 200 python -u bench/decode_bench.py --batches $B --decode-only 40 > gpurun_out/ab3_${name}_$B.log 2>&1 || exit 1
    echo "$name B=$B $(grep -h '^{' gpurun_out/ab3_${name}_$B.log | grep -o '"decode_ms_per_step": [0-9.]*')"
  done
}
run head_old KCA_KERNEL_LIB=$PWD/ab/libkca_kernels_head.so KCA_DECODE_SPLIT_POLICY=wgs1024 || exit 1
run new_old KCA_DECODE_SPLIT_POLICY=wgs1024 || exit 1
run new_256 KCA_DECODE_WGS=256 || exit 1
run new_512 KCA_DECODE_WGS=512 || exit 1
run new_1024 KCA_DECODE_WGS=1024 || exit 1
run head_old_serial KCA_KERNEL_LIB=$PWD/ab/libkca_kernels_head.so KCA_DECODE_SPLIT_POLICY=wgs1024 KCA_DECODE_PAR_MLP=0 || exit 1
run new_256_serial KCA_DECODE_PAR_MLP=0 || exit 1
