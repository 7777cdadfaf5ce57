# GPT-J decode: split workgroup target 256 vs 1024, interleaved repeats (bench/decode_bench.py).
mkdir -p gpurun_out
for rep in 1 2; do
  for W in 256 1024; do
    for B in 1 8 32; do
      KCA_DECODE_WGS=$W timeout -k 10 200 python -u bench/decode_bench.py --batches $B --decode-only 40 > gpurun_out/ab4_${W}_${B}_$rep.log 2>&1 || exit 1
      echo "W=$W B=$B rep=$rep $(grep -h '^{' gpurun_out/ab4_${W}_${B}_$rep.log | grep -o '"decode_ms_per_step": [0-9.]*')"
    done
  done
done
