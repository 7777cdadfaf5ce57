# round-4 batch 34: GPT-J B=1 decode timeline after the step descriptors
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
rm -rf gpurun_out/dec_tl
bash tools/gpu_decode_timeline.sh || { tail -20 gpurun_out/dec_tl.log; exit 1; }
f=$(find gpurun_out/dec_tl -name '*kernel_trace.csv' | head -1)
python3 tools/timeline.py "$f" --step-kernel "void ln_rows_kernel<2, true>" --steps 10 --show 12 > gpurun_out/dec_tl_r4_desc.txt 2>&1
cat gpurun_out/dec_tl_r4_desc.txt
