# K-split sweep of the batched-decode MFMA GEMM on the fused-layer shapes (forced --ks)
set -o pipefail
for ks in 1 2 3 4 6 8; do
  timeout -k 10 120 python -u bench/mm_bench.py --variants mfma --ks $ks --ms 8,32 \
    --shapes gptj.qkv_fcin,gptj.out_fcout,gptj.out,bloom8.qkv,bloom8.out,bloom8.fc_in,bloom8.fc_out,neox.qkv,neox.fc_in,neox.fc_out \
    > gpurun_out/ks_sweep_$ks.jsonl 2>/dev/null || exit 2
done
