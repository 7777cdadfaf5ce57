#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
KCA_AR_GATHER=0 timeout -k 10 120 python -u tools/debug/tp_hang.py > gpurun_out/r3_dbg_nogather.log 2>&1
echo "nogather rc=$?"
timeout -k 10 120 python -u tools/debug/tp_hang.py > gpurun_out/r3_dbg_gather.log 2>&1
echo "gather rc=$?"
