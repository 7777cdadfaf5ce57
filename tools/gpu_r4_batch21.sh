# round-4 batch 21: in-kernel stamps of the fused decode layer kernel in a real GPT-J B=1 step
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u bench/decode_layer_stamps.py --steps 8 2> gpurun_out/dec_stamps.err | tee gpurun_out/dec_layer_stamps_r4.jsonl || { tail -20 gpurun_out/dec_stamps.err; exit 1; }
