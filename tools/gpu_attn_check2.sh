set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "attention or unet_padded" -x -q --timeout 120 --timeout-method thread > gpurun_out/attn_tests.log 2>&1 || { tail -30 gpurun_out/attn_tests.log; exit 1; }
tail -2 gpurun_out/attn_tests.log
SHAPES="gptj,neox20b,bloom_tp8,gpt2,sd_64_pad64,d160_4k" bash tools/gpu_attn_ab.sh
