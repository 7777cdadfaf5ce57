# round-4 batch 31: GPT-J step kernel split refresh (GEMM-side gradient accumulation), plain-run number
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
( cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/step_prof2 -o step -- python3 $GRAFT_REPO_ROOT/bench.py --steps 3 --warmup 2 --sd 0 --extra off --bloom-tp off > $GRAFT_REPO_ROOT/gpurun_out/step_prof2.log 2>&1 ) || { tail -20 gpurun_out/step_prof2.log; exit 1; }
f=$(find gpurun_out/step_prof2 -name '*kernel_trace.csv' | head -1)
python3 tools/step_window.py "$f" --first 2 --last 5 > gpurun_out/step_split_r4b.txt 2>&1
head -30 gpurun_out/step_split_r4b.txt
