# rocprofv3 kernel trace of SD-1.5 txt2img (batch 8, 512 px, 10 LMS steps) for the per-kernel split
set -o pipefail
export TMPDIR=/tmp
mkdir -p $GRAFT_REPO_ROOT/gpurun_out
cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/sd_prof -o sd -- python3 $GRAFT_REPO_ROOT/bench/sd_bench.py --mode infer --steps 1 --warmup 1 --infer-steps 10 > $GRAFT_REPO_ROOT/gpurun_out/sd_prof.log 2>&1
