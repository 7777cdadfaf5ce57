# round-4 batch 18: wgrad GEMM + fp32 accumulation (split vs hipBLASLt fp32-output in place), block GEMM efficiency
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u bench/wgrad_accum_bench.py --layer-gemms > gpurun_out/wgrad_accum_r4.jsonl 2> gpurun_out/wgrad_accum_r4.err || { tail -20 gpurun_out/wgrad_accum_r4.err; exit 1; }
cat gpurun_out/wgrad_accum_r4.jsonl
