# rocprofv3 kernel trace of GPT-J decode (B=1, decode-only) for tools/timeline.py
set -o pipefail
export TMPDIR=/tmp
mkdir -p $GRAFT_REPO_ROOT/gpurun_out
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/dec_tl -o dec -- python3 $GRAFT_REPO_ROOT/bench/decode_bench.py --batches ${B:-1} --decode-only 40 > $GRAFT_REPO_ROOT/gpurun_out/dec_tl.log 2>&1
