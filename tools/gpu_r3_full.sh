#!/bin/bash
# full GPU suite + smoke + shared-GPU 2-rank bench rehearsal
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 240 --timeout-method thread \
  > gpurun_out/r3_gpu_tests.log 2>&1
echo "tests rc=$?"
tail -5 gpurun_out/r3_gpu_tests.log
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r3_smoke.log 2>&1 || exit 2
KCA_BENCH_SHARED_GPU=1 timeout -k 10 300 python -u bench.py --gpus 2 --steps 2 --warmup 1 --layers 2 --hidden 1024 \
  --heads 4 --seq 512 --micro-batch 2 --gas 2 --sd 0 --bloom-layers 2 --bloom-batches 1,4 --tunableop off \
  > gpurun_out/r3_shared_bench.out 2> gpurun_out/r3_shared_bench.err
echo "shared bench rc=$?"
