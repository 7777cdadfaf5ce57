#!/bin/bash
# Sampler change check on one GPU: draw identity against the previous library, the sampler tests,
# segment stamps and per-mode kernel times (tools/sampler_profile.py).
# Needs (built on the CPU first): ab/libkca_kernels_old.so -- the baseline commit's kernels, e.g.
#   git worktree add ab/oldtree <commit> && (cd ab/oldtree && python tools/build_ext.py) &&
#   cp ab/oldtree/kubernetes_cloud_amd/_lib/libkca_kernels.so ab/libkca_kernels_old.so
# -- and ab/libkca_kernels_stamps.so (python tools/build_ext.py --stamps).
set -o pipefail
cd /root/repo && mkdir -p gpurun_out/samp && export TMPDIR=/tmp
KCA_KERNEL_LIB=$PWD/ab/libkca_kernels_old.so timeout -k 10 120 python tools/sampler_identity.py --out gpurun_out/samp/old.pt &&
timeout -k 10 120 python tools/sampler_identity.py --out gpurun_out/samp/new.pt &&
python tools/sampler_identity.py --compare gpurun_out/samp/old.pt gpurun_out/samp/new.pt > gpurun_out/samp/identity.txt; echo "identity rc=$?" >> gpurun_out/samp/identity.txt
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_decode_gpu.py -k sample > gpurun_out/samp/tests.txt 2>&1 &&
KCA_KERNEL_LIB=$PWD/ab/libkca_kernels_stamps.so timeout -k 10 120 python tools/sample_stamps.py --modes greedy,topk10,topk50,topk50_topp0.95 > gpurun_out/samp/stamps.txt 2>&1 &&
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/samp/prof -o s -- python3 tools/sample_bench.py > gpurun_out/samp/bench.txt 2>&1 &&
python tools/sampler_profile.py $(ls gpurun_out/samp/prof/*/s_kernel_trace.csv gpurun_out/samp/prof/s_kernel_trace.csv 2>/dev/null | head -1) > gpurun_out/samp/profile.md
