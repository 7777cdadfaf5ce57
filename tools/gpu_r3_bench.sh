#!/bin/bash
# default bench.py exactly as the driver runs it at N=1 (headline + secondaries), then a kernel-stats
# profile of txt2img with the round-3 defaults
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
s=$(date +%s)
timeout -k 10 900 python -u bench.py > gpurun_out/r3_bench.out 2> gpurun_out/r3_bench.err || { echo "bench rc=$?"; tail -20 gpurun_out/r3_bench.err; exit 2; }
echo "bench wall $(( $(date +%s) - s )) s"
tail -c 3000 gpurun_out/r3_bench.out
cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/sd_prof_r3b -o sd -- python3 $GRAFT_REPO_ROOT/bench/sd_bench.py --mode infer --steps 1 --warmup 1 --infer-steps 10 > $GRAFT_REPO_ROOT/gpurun_out/sd_prof_r3b.log 2>&1 || exit 4
echo profiled
