#!/bin/bash
# Same-box interleaved A/B of one command under two environments (the only A/B runner; one-off
# scripts of rounds 1-3 live in git history). Results: gpurun_out/<name>_{A,B}_<rep>.out
#   tools/gpu_ab.sh <name> <reps> "<env A>" "<env B>" <timeout s> <command...>
#   e.g. tools/gpu_ab.sh fuse_res 2 "KCA_SD_FUSE_RES=0" "KCA_SD_FUSE_RES=1" 300 python -u bench/sd_bench.py --mode infer --steps 4
# A pytest prelude can be given as GPU_AB_TESTS="tests/a.py tests/b.py" (runs first, stops on failure).
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
name=$1; reps=$2; envA=$3; envB=$4; tmo=$5; shift 5
if [ -n "$GPU_AB_TESTS" ]; then
  timeout -k 10 600 python -u -m pytest $GPU_AB_TESTS -x -q --timeout 200 --timeout-method thread \
    > gpurun_out/${name}_tests.log 2>&1 || { tail -30 gpurun_out/${name}_tests.log; exit 1; }
  tail -2 gpurun_out/${name}_tests.log
fi
for rep in $(seq 1 "$reps"); do
  for arm in A B; do
    if [ $arm = A ]; then e=$envA; else e=$envB; fi
    env $e timeout -k 10 "$tmo" "$@" > gpurun_out/${name}_${arm}_${rep}.out 2> gpurun_out/${name}_${arm}_${rep}.err || {
      echo "arm $arm rep $rep failed ($?)"; tail -20 gpurun_out/${name}_${arm}_${rep}.err; exit 2; }
    echo "== $arm ($e) rep $rep"; grep -v "amdgpu.ids" gpurun_out/${name}_${arm}_${rep}.out | tail -8
  done
done
