cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for v in 0 1; do
KCA_MULTI_ACCUM=$v timeout -k 10 300 python -u -m pytest tests/test_multirank_gpu.py -k zero_stages -x -q --timeout 250 --timeout-method thread > gpurun_out/accdbg_$v.log 2>&1
echo "MULTI_ACCUM=$v rc=$?"; grep -E "passed|failed|AssertionError:" gpurun_out/accdbg_$v.log | head -3
done
