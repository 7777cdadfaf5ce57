# Decode attention A/B, cold caches: the committed kernel library (ab/libkca_kernels_head.so)
# against the working tree's, same box (bench/decode_attn_bench.py --cold).
mkdir -p gpurun_out
ARGS="--cold --ctx ${CTX:-600 2048} --batch ${BATCH:-1 8 32} --chunk ${CHUNKS:-32 64 128 256 1024}"
KCA_KERNEL_LIB=$PWD/ab/libkca_kernels_head.so timeout -k 10 300 python -u bench/decode_attn_bench.py $ARGS > gpurun_out/dattn_ab_head.log 2>&1 || exit 1
timeout -k 10 300 python -u bench/decode_attn_bench.py $ARGS > gpurun_out/dattn_ab_new.log 2>&1 || exit 1
echo done
