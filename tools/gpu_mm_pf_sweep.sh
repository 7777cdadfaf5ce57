# Weight-chunks-in-flight (KCA_MM_PF) x K-chunk (KCA_MM_KC) sweep of the batched-decode MFMA GEMM,
# hipBLASLt beside it, M = 8 / 32 / 64
set -o pipefail
mkdir -p gpurun_out/mm_pf_sweep
S=gptj.qkv_fcin,gptj.out_fcout,bloom8.qkv,bloom8.out,bloom8.fc_in,bloom8.fc_out,neox.qkv,neox.fc_in,neox.fc_out
for kc in 256 128; do
  for pf in 1 2 3; do
    KCA_MM_KC=$kc KCA_MM_PF=$pf timeout -k 10 150 python -u bench/mm_bench.py --variants mfma --ms 8,32,64 \
      --shapes $S > gpurun_out/mm_pf_sweep/kc${kc}_pf$pf.jsonl 2>/dev/null || exit 2
  done
done
timeout -k 10 150 python -u bench/mm_bench.py --variants blas --ms 8,32,64 --shapes $S \
  > gpurun_out/mm_pf_sweep/blas.jsonl 2>/dev/null || exit 2
