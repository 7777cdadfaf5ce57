#!/bin/bash
# SD fused-step kernels on MI355X: numerics tests, the DreamBooth entry point, and DreamBooth / txt2img A/B.
set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_kernels_gpu.py -k "sd_fused" tests/test_entrypoints_gpu.py > gpurun_out/sd_tests.log 2>&1 && \
KCA_SD_FUSED_TRAIN=0 timeout -k 10 400 python -u bench/sd_bench.py --mode train --steps 10 > gpurun_out/sd_train_unfused.log 2>&1 && \
timeout -k 10 400 python -u bench/sd_bench.py --mode train --steps 10 > gpurun_out/sd_train_fused.log 2>&1 && \
KCA_SD_FUSED_STEP=0 timeout -k 10 400 python -u bench/sd_bench.py --mode infer --steps 2 > gpurun_out/sd_infer_unfused.log 2>&1 && \
timeout -k 10 400 python -u bench/sd_bench.py --mode infer --steps 2 > gpurun_out/sd_infer_fused.log 2>&1
