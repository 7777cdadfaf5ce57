# TunableOp search for the GPT-J step's GEMMs at the headline micro-batch 16 (the shipped table was tuned at
# micro-batch 8: 16384-token shapes), then a same-box A/B of the headline with the old vs the new table
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
cp tuning/tunableop_results.csv gpurun_out/tunableop_gptj_mb16.csv
timeout -k 10 600 python -u bench.py --steps 2 --warmup 1 --sd 0 --extra off --bloom-tp off --tunableop tune --tunableop-file $PWD/gpurun_out/tunableop_gptj_mb16.csv > gpurun_out/tune_gptj.json 2> gpurun_out/tune_gptj.err || { tail -20 gpurun_out/tune_gptj.err; exit 1; }
grep -c "" gpurun_out/tunableop_gptj_mb16.csv
for f in tuning/tunableop_results.csv gpurun_out/tunableop_gptj_mb16.csv tuning/tunableop_results.csv gpurun_out/tunableop_gptj_mb16.csv; do
  timeout -k 10 400 python -u bench.py --steps 5 --warmup 2 --sd 0 --extra off --bloom-tp off --tunableop use --tunableop-file $PWD/$f 2>/dev/null | tail -1 | cut -c1-140
  echo "  ($f)"
done
