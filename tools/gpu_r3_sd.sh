#!/bin/bash
# SD attention rowsum variant: tests + attention microbench A/B + txt2img A/B
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_attention_masks_gpu.py -x -v --timeout 200 --timeout-method thread \
  > gpurun_out/r3_sd_tests.log 2>&1 || { tail -30 gpurun_out/r3_sd_tests.log; exit 1; }
tail -2 gpurun_out/r3_sd_tests.log
for rep in 1 2; do
for rs in 0 1; do
KCA_SD_ROWSUM_COL=$rs timeout -k 10 300 python -u bench/sd_bench.py --mode infer --steps 4 > gpurun_out/r3_sd_rs${rs}_${rep}.jsonl 2> gpurun_out/r3_sd_rs${rs}_${rep}.err || exit 2
echo "rowsum=$rs rep=$rep $(cat gpurun_out/r3_sd_rs${rs}_${rep}.jsonl)"
done
done
