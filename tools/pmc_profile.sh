#!/bin/bash
# Counter profile of the hand-written gfx950 kernels (bench/kernel_pmc.py), one
# rocprofv3 pass per counter group (gfx950 slot limits: <=8 SQ, <=4 TCC with
# FETCH_SIZE=3 / WRITE_SIZE=2, <=2 GRBM), plus one kernel-trace pass for
# durations. Summarise with: python tools/pmc_summary.py gpurun_out/pmc
# Run on the GPU box: gpurun -- bash tools/pmc_profile.sh
set -e
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/pmc
mkdir -p $OUT
CASES=${CASES:-attn_gptj,attn_sd64,layernorm_gptj,groupnorm_nhwc_sd,geglu_sd,xent_gptj,adamw_512m,gemv_fcin_m1,decode_attn_b32}
run() {  # run <tag> <rocprofv3 args...>
  tag=$1; shift
  timeout -s KILL 240 rocprofv3 "$@" -d $OUT/$tag -o $tag --output-format csv -- \
    python3 bench/kernel_pmc.py --cases $CASES --out $OUT/cases.json > $OUT/$tag.log 2>&1
  echo "[pmc_profile] pass $tag done"
}
run trace --kernel-trace --stats
run sqA --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE
run fetch --pmc FETCH_SIZE GRBM_GUI_ACTIVE SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS
run write --pmc WRITE_SIZE GRBM_GUI_ACTIVE
