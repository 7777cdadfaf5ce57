# round-4 batch 6: GPT-J headline step (LM head TN dgrad, LN bwd prefetch): bench number, kernel split, attention counters
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u bench.py --steps 5 --warmup 2 --sd 0 --extra off --bloom-tp off > gpurun_out/bench_r4_gptj.json 2> gpurun_out/bench_r4_gptj.err || { tail -20 gpurun_out/bench_r4_gptj.err; exit 1; }
tail -1 gpurun_out/bench_r4_gptj.json
(cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/step_prof_r4 -o step -- python3 $GRAFT_REPO_ROOT/bench.py --steps 3 --warmup 2 --sd 0 --extra off --bloom-tp off > $GRAFT_REPO_ROOT/gpurun_out/step_prof_r4.log 2>&1) || { echo "step prof failed"; tail -5 gpurun_out/step_prof_r4.log; exit 1; }
python tools/step_window.py gpurun_out/step_prof_r4/step_kernel_trace.csv --first 2 --last 5 | head -30
CASES=attn_gptj bash tools/pmc_profile.sh > gpurun_out/pmc_r4.log 2>&1 || { tail -10 gpurun_out/pmc_r4.log; exit 1; }
python tools/pmc_summary.py gpurun_out/pmc | head -12
timeout -k 10 400 python -u bench/serving_bench.py > gpurun_out/serving_r4_v3.jsonl 2>gpurun_out/serving_r4_v3.err || { tail -20 gpurun_out/serving_r4_v3.err; exit 1; }
cat gpurun_out/serving_r4_v3.jsonl
