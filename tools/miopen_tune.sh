#!/bin/bash
# Re-tune MIOpen's convolution solvers for the SD-1.5 bench shapes on an MI355X
# and refresh tuning/miopen/ (see kubernetes_cloud_amd/utils/miopen.py).
# Run on the GPU box: gpurun -- bash tools/miopen_tune.sh ; then copy
# gpurun_out/miotune/db/*.txt into tuning/miopen/.
set -e
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/miotune
mkdir -p $OUT/db $OUT/cache
cp tuning/miopen/*.txt $OUT/db/ 2>/dev/null || true
export MIOPEN_USER_DB_PATH=$PWD/$OUT/db MIOPEN_CUSTOM_CACHE_DIR=$PWD/$OUT/cache MIOPEN_FIND_ENFORCE=3
timeout -k 10 300 python -u tools/sd_breakdown.py > $OUT/infer.log 2>&1
timeout -k 10 500 python -u bench/sd_bench.py --mode train --steps 2 --warmup 1 > $OUT/train.log 2>&1
echo "[miopen_tune] done"
