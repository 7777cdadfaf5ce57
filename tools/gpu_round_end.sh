# Round-end rehearsal on one MI355X: GPU test suite, smoke(), bench.py (GPT-J + SD), each step bounded.
set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/re_tests.log 2>&1 || { tail -30 gpurun_out/re_tests.log; exit 1; }
tail -1 gpurun_out/re_tests.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/re_smoke.log 2>&1 || { tail -20 gpurun_out/re_smoke.log; exit 1; }
tail -1 gpurun_out/re_smoke.log
timeout -k 10 600 python -u bench.py > gpurun_out/re_bench.log 2>&1 || { tail -20 gpurun_out/re_bench.log; exit 1; }
grep "^\[bench\]" gpurun_out/re_bench.log
grep "^{" gpurun_out/re_bench.log
