#!/bin/bash
# ZeRO stages at world 2 on one GPU, TP engine (shm control channel), shared-GPU bench record
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 500 python -u -m pytest -x -v --timeout 360 --timeout-method thread \
  tests/test_multirank_gpu.py::test_zero_stages_world2_on_gpu_match tests/test_tp_engine_gpu.py \
  tests/test_custom_ar_gpu.py > gpurun_out/r3_zero.log 2>&1 || exit 2
KCA_BENCH_SHARED_GPU=1 timeout -k 10 300 python -u bench.py --gpus 2 --steps 2 --warmup 1 --layers 2 --hidden 1024 \
  --heads 4 --seq 512 --micro-batch 2 --gas 2 --sd 0 --bloom-layers 2 --bloom-batches 1,4 --tunableop off \
  > gpurun_out/r3_shared_bench.out 2> gpurun_out/r3_shared_bench.err || exit 3
echo done
