# rocprofv3 kernel split of the SD-1.5 DreamBooth training step (8 instance + 8 class, 512 px)
set -o pipefail
export TMPDIR=/tmp
mkdir -p $GRAFT_REPO_ROOT/gpurun_out
cd /tmp && timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/sdt_prof -o sdt -- python3 $GRAFT_REPO_ROOT/bench/sd_bench.py --mode train --steps 4 --warmup 2 > $GRAFT_REPO_ROOT/gpurun_out/sdt_prof.log 2>&1
