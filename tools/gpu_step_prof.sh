# rocprofv3 kernel split of the default bench.py GPT-J step (mb16 x GAS2), no SD / BLOOM phases
set -o pipefail
export TMPDIR=/tmp
mkdir -p $GRAFT_REPO_ROOT/gpurun_out
cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/step_prof -o step -- python3 $GRAFT_REPO_ROOT/bench.py --steps 3 --warmup 2 --sd 0 > $GRAFT_REPO_ROOT/gpurun_out/step_prof.log 2>&1
