# GPT-J decode A/B: committed library (head) vs working tree with the split-K fan-in off / on
# (nt weight loads in both new arms); decode GPU tests first; interleaved repeats.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_decode_gpu.py tests/test_kernels_gpu.py -k "decode or sampl or gemv or skinny" -x -q --timeout 120 --timeout-method thread > gpurun_out/decode_tests.log 2>&1 || { tail -30 gpurun_out/decode_tests.log; exit 1; }
tail -1 gpurun_out/decode_tests.log
: > gpurun_out/nt_ab.log
for rep in 1 2; do
  for arm in head new0 new1; do
    for B in ${BATCHES:-1 8 32}; do
      case $arm in
        head) env="KCA_KERNEL_LIB=$PWD/ab/libkca_kernels_head.so KCA_DECODE_FANIN=1";;
        new0) env="KCA_DECODE_FANIN=0";;
        new1) env="KCA_DECODE_FANIN=1";;
      esac
      env $env timeout -k 10 200 python -u bench/decode_bench.py --batches $B --decode-only 40 > gpurun_out/nt_${arm}_${B}_$rep.log 2>&1 || exit 1
      echo "arm=$arm B=$B rep=$rep $(grep -h '^{' gpurun_out/nt_${arm}_${B}_$rep.log | grep -o '"decode_ms_per_step": [0-9.]*')" | tee -a gpurun_out/nt_ab.log
    done
  done
done
