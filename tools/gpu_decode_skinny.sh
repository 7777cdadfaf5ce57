# GPT-J decode at small batch: hipBLASLt (default for M >= 2) vs the skinny GEMV kernel with nt weight loads
mkdir -p gpurun_out
: > gpurun_out/skinny_ab.log
for rep in 1 2; do
  for X in 1 2; do
    for B in 1 2 4; do
      KCA_SKINNY_MAX_M=$X timeout -k 10 200 python -u bench/decode_bench.py --batches $B --decode-only 40 > gpurun_out/sk_${X}_${B}_$rep.log 2>&1 || exit 1
      echo "max_m=$X B=$B rep=$rep $(grep -h '^{' gpurun_out/sk_${X}_${B}_$rep.log | grep -o '"decode_ms_per_step": [0-9.]*')" | tee -a gpurun_out/skinny_ab.log
    done
  done
done
