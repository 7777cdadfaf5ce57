# rocprofv3 kernel trace of the BLOOM-176B TP=8 rank-0 emulation (the deployment's launch structure:
# matrix-core layer + fused all-reduce tails over a rank-local custom all-reduce) at batch ${B:-8},
# split per step by tools/rocpd_split.py (no hipBLASLt / at::native / standalone LN
# inside the layer loop)
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace -d $R/gpurun_out/bloom_tl -o bloom -- python3 $R/bench/decode_suite.py --models bloom8 --batches ${B:-8} --dtypes ${DT:-bf16} > $R/gpurun_out/bloom_tl.log 2>&1 || exit 1
db=$(ls $R/gpurun_out/bloom_tl/*.db 2>/dev/null | head -1)
[ -n "$db" ] || db=$(find $R/gpurun_out/bloom_tl -name "*.db" | head -1)
python3 $R/tools/rocpd_split.py "$db" --last-steps 10 --step-kernel sample_ > $R/gpurun_out/bloom_tl_split.txt
