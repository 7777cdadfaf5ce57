# round-4 batch 16: MIOpen re-tune for the current SD step (DreamBooth fwd/bwd/wrw + txt2img UNet/VAE shapes),
# DreamBooth / txt2img with the shipped db vs the re-tuned one
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
bash tools/miopen_tune.sh > gpurun_out/miotune.log 2>&1 || { tail -5 gpurun_out/miotune.log; tail -5 gpurun_out/miotune/infer.log; exit 1; }
ls -la gpurun_out/miotune/db
for db in $PWD/tuning/miopen $PWD/gpurun_out/miotune/db $PWD/tuning/miopen $PWD/gpurun_out/miotune/db; do
  MIOPEN_USER_DB_PATH=$db timeout -k 10 300 python -u bench/sd_bench.py --mode train --steps 10 --warmup 3 2>/dev/null | tail -1 | cut -c1-120; echo "  ($db)"
done
for db in $PWD/tuning/miopen $PWD/gpurun_out/miotune/db; do
  MIOPEN_USER_DB_PATH=$db timeout -k 10 300 python -u bench/sd_bench.py --mode infer --steps 3 --warmup 1 2>/dev/null | tail -1 | cut -c1-120; echo "  ($db)"
done
