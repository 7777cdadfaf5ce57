# GPT-J decode: split-K fan-in in the attention kernel vs the separate combine kernel (KCA_DECODE_FANIN=0),
# same library, interleaved repeats; decode GPU tests first.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_decode_gpu.py tests/test_kernels_gpu.py -k "decode or sampl" -x -q --timeout 120 --timeout-method thread > gpurun_out/decode_tests.log 2>&1 || { tail -30 gpurun_out/decode_tests.log; exit 1; }
tail -2 gpurun_out/decode_tests.log
: > gpurun_out/fanin_ab.log
for rep in 1 2; do
  for F in 0 1; do
    for B in ${BATCHES:-1 8 32}; do
      KCA_DECODE_FANIN=$F timeout -k 10 200 python -u bench/decode_bench.py --batches $B --decode-only 40 > gpurun_out/fanin_${F}_${B}_$rep.log 2>&1 || exit 1
      echo "fanin=$F B=$B rep=$rep $(grep -h '^{' gpurun_out/fanin_${F}_${B}_$rep.log | grep -o '"decode_ms_per_step": [0-9.]*')" | tee -a gpurun_out/fanin_ab.log
    done
  done
done
