# GPT-J decode B=1: separate LN rows kernel (KCA_DECODE_LN_SPLIT=1) vs LN in the QKV GEMV prologue (0)
mkdir -p gpurun_out
: > gpurun_out/lnsplit_ab.log
for rep in 1 2 3; do
  for S in 1 0; do
    KCA_DECODE_LN_SPLIT=$S timeout -k 10 200 python -u bench/decode_bench.py --batches ${B:-1} --decode-only 40 > gpurun_out/ln_${S}_$rep.log 2>&1 || exit 1
    echo "ln_split=$S rep=$rep $(grep -h '^{' gpurun_out/ln_${S}_$rep.log | grep -o '"decode_ms_per_step": [0-9.]*')" | tee -a gpurun_out/lnsplit_ab.log
  done
done
