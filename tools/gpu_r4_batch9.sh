# round-4 batch 9: GPU suite, DreamBooth (shared silu(temb), VAE conv_in fold, native quick GELU) attribution + split, txt2img
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/gpu_suite_r4b.log 2>&1 || { tail -40 gpurun_out/gpu_suite_r4b.log; exit 1; }
tail -2 gpurun_out/gpu_suite_r4b.log
timeout -k 10 300 python -u bench/sd_bench.py --mode train --steps 3 --warmup 2 --attrib > gpurun_out/sdt_attrib_r4d.json 2> gpurun_out/sdt_attrib_r4d.err || { tail -20 gpurun_out/sdt_attrib_r4d.err; exit 1; }
grep -A30 "attrib\]" gpurun_out/sdt_attrib_r4d.err | head -32
(cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/sdt_prof_r4c -o sdt -- python3 $GRAFT_REPO_ROOT/bench/sd_bench.py --mode train --steps 4 --warmup 2 > $GRAFT_REPO_ROOT/gpurun_out/sdt_prof_r4c.log 2>&1) || { echo "train prof failed"; exit 1; }
for i in 1 2; do timeout -k 10 300 python -u bench/sd_bench.py --mode train --steps 10 --warmup 3 2>/dev/null | tail -1; done
timeout -k 10 300 python -u bench/sd_bench.py --mode infer --steps 3 --warmup 1 2>/dev/null | tail -1
