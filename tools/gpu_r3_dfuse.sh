#!/bin/bash
# DIAGNOSTIC: dual GEMV cost of the LN tail (diag 1) and of the arrival (diag 2); outputs are wrong in B
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
bash tools/gpu_ab.sh ddiag1 2 "KCA_DUAL_DIAG=0" "KCA_DUAL_DIAG=1" 300 \
  python -u bench/decode_bench.py --batches 1 --decode-only 48 &&
bash tools/gpu_ab.sh ddiag2 2 "KCA_DUAL_DIAG=0" "KCA_DUAL_DIAG=2" 300 \
  python -u bench/decode_bench.py --batches 1 --decode-only 48
