#!/bin/bash
# attention max-column variant: tests, kernel microbench, txt2img A/B
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_attention_masks_gpu.py tests/test_unet_fusions_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/mc_tests.log 2>&1 || { tail -30 gpurun_out/mc_tests.log; exit 1; }
tail -2 gpurun_out/mc_tests.log
timeout -k 10 300 python -u bench/attn_bench.py --no-sdpa --fwd-only --shapes sd_64_pad48_rs,sd_64_pad48_mc,sd_64_pad48_rs,sd_64_pad48_mc,sd_cross > gpurun_out/mc_attn.jsonl 2>&1 || { tail -5 gpurun_out/mc_attn.jsonl; exit 2; }
grep shape gpurun_out/mc_attn.jsonl
bash tools/gpu_ab.sh sd_mc 2 "KCA_SD_MAX_COL=0" "KCA_SD_MAX_COL=1" 300 python -u bench/sd_bench.py --mode infer --steps 4
