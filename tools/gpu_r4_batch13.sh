# round-4 batch 13: the N=2 bench path rehearsed as 2 ranks on one GPU (ZeRO-1, shrunk GPT-J), deferred param
# all-gather on vs off: same losses; plus the gloo-free unit tests of the engine on the GPU
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
for arm in 1 0; do
  KCA_DEFER_ALLGATHER=$arm KCA_BENCH_SHARED_GPU=1 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 2960$arm bench.py --gpus 2 --steps 3 --warmup 1 --layers 4 --micro-batch 4 --sd 0 --extra off --bloom-tp off > gpurun_out/shared2_defer$arm.json 2> gpurun_out/shared2_defer$arm.err || { tail -20 gpurun_out/shared2_defer$arm.err; exit 1; }
  echo "defer=$arm $(grep -h 'loss=' gpurun_out/shared2_defer$arm.err | tail -1)"
done
