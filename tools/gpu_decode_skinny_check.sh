timeout -k 10 300 python -u -m pytest tests/test_decode_gpu.py -k "skinny" -x -q --timeout 120 --timeout-method thread > gpurun_out/skinny_tests.log 2>&1 || { tail -30 gpurun_out/skinny_tests.log; exit 1; }
tail -1 gpurun_out/skinny_tests.log
bash tools/gpu_decode_skinny.sh
