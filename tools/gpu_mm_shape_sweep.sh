# Workgroup-shape sweep of the batched-decode MFMA GEMM: 16-row tiles per wave (KCA_MM_NR), K chunk
# (KCA_MM_KC), waves per workgroup (KCA_MM_WV) -- wider N blocks re-read the activation fewer times
set -o pipefail
mkdir -p gpurun_out/mm_shape_sweep
S=gptj.qkv_fcin,gptj.out_fcout,bloom8.qkv,bloom8.out,bloom8.fc_in,bloom8.fc_out,neox.qkv,neox.fc_in,neox.fc_out
for cfg in 2:128:4 2:256:4 1:128:8 1:256:8 2:128:8; do
  IFS=: read nr kc wv <<< "$cfg"
  KCA_MM_NR=$nr KCA_MM_KC=$kc KCA_MM_WV=$wv timeout -k 10 150 python -u bench/mm_bench.py --variants mfma --ms 8,32,64 \
    --shapes $S > gpurun_out/mm_shape_sweep/nr${nr}_kc${kc}_wv${wv}.jsonl 2>/dev/null || exit 2
done
