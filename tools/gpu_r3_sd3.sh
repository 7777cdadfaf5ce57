#!/bin/bash
# SD inference round-3 fusions: tests, upsampler microbench, txt2img A/B (all new paths off vs defaults)
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python -u bench/upsample_conv_bench.py > gpurun_out/r3_upconv2.jsonl 2> gpurun_out/r3_upconv2.err || { tail -5 gpurun_out/r3_upconv2.err; exit 5; }
cat gpurun_out/r3_upconv2.jsonl
GPU_AB_TESTS="tests/test_unet_fusions_gpu.py tests/test_kernels_gpu.py tests/test_entrypoints_gpu.py" bash tools/gpu_ab.sh sd_up 2 \
  "KCA_SD_PHASE_UP=0 KCA_SD_CAT_GN=0 KCA_SD_TEMB_BATCH=0 KCA_SD_CTX_KV=0" "KCA_SD_PHASE_UP=1" 300 python -u bench/sd_bench.py --mode infer --steps 4
