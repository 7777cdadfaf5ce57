# TP=2 decode timeline, two ranks sharing the one GPU (custom xGMI all-reduce kernel over IPC, shared-memory
# control channel, one-step lookahead): rank 0 under rocprofv3 kernel trace, rank 1 plain. No launcher re-exec.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0 KCA_BENCH_SHARED_GPU=1 MASTER_ADDR=127.0.0.1 MASTER_PORT=29611 WORLD_SIZE=2 LOCAL_WORLD_SIZE=2
R=$GRAFT_REPO_ROOT
(RANK=1 LOCAL_RANK=1 timeout -k 10 400 python3 $R/bench/bloom_tp_bench.py --layers 4 --batches 1 --new-tokens 64 > $R/gpurun_out/tp2_r1.log 2>&1) &
P1=$!
(cd /tmp && RANK=0 LOCAL_RANK=0 timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/tp2_tl -o tp -- python3 $R/bench/bloom_tp_bench.py --layers 4 --batches 1 --new-tokens 64 > $R/gpurun_out/tp2_r0.log 2>&1)
rc0=$?
wait $P1
rc1=$?
tail -3 gpurun_out/tp2_r0.log
[ $rc0 -eq 0 ] && [ $rc1 -eq 0 ]
