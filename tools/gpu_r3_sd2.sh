#!/bin/bash
# SD inference changes: 48-wide narrow heads + hipBLASLt bias/residual epilogue. Tests, kernel A/B,
# txt2img three-arm A/B, then a kernel-stats profile of txt2img.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_attention_masks_gpu.py tests/test_gemm_lt_gpu.py tests/test_kernels_gpu.py \
  tests/test_entrypoints_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r3_sd2_tests.log 2>&1 \
  || { tail -30 gpurun_out/r3_sd2_tests.log; exit 1; }
tail -2 gpurun_out/r3_sd2_tests.log
timeout -k 10 300 python -u bench/attn_bench.py --no-sdpa --fwd-only --shapes sd_64_pad64,sd_64_pad48,sd_64_pad64,sd_64_pad48 > gpurun_out/r3_narrow_attn.jsonl 2>&1 || exit 2
grep shape gpurun_out/r3_narrow_attn.jsonl
for rep in 1 2; do
  for arm in "KCA_SD_NARROW_HEADS=0 KCA_SD_FUSE_RES=0" "KCA_SD_NARROW_HEADS=1 KCA_SD_FUSE_RES=0" "KCA_SD_NARROW_HEADS=1 KCA_SD_FUSE_RES=1"; do
    tag=$(echo $arm | tr -dc '01')
    env $arm timeout -k 10 300 python -u bench/sd_bench.py --mode infer --steps 4 > gpurun_out/r3_sd2_${tag}_${rep}.jsonl 2> gpurun_out/r3_sd2_${tag}_${rep}.err || exit 3
    echo "$arm rep $rep $(cat gpurun_out/r3_sd2_${tag}_${rep}.jsonl)"
  done
done
timeout -k 10 300 python -u bench/upsample_conv_bench.py > gpurun_out/r3_upconv.jsonl 2> gpurun_out/r3_upconv.err || { tail -5 gpurun_out/r3_upconv.err; exit 5; }
cat gpurun_out/r3_upconv.jsonl
export TMPDIR=/tmp
cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/sd_prof_r3 -o sd -- python3 $GRAFT_REPO_ROOT/bench/sd_bench.py --mode infer --steps 1 --warmup 1 --infer-steps 10 > $GRAFT_REPO_ROOT/gpurun_out/sd_prof_r3.log 2>&1 || exit 4
ls -R $GRAFT_REPO_ROOT/gpurun_out/sd_prof_r3 | head
