# round-4 SD batch: DreamBooth eager-kernel attribution, DreamBooth kernel split (48-wide training heads),
# txt2img kernel split (wide VAE flash), both benches with the VAE / narrow-training A/B knobs
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u bench/sd_bench.py --mode train --steps 3 --warmup 2 --attrib > gpurun_out/sdt_attrib_r4.json 2> gpurun_out/sdt_attrib_r4.err || { tail -20 gpurun_out/sdt_attrib_r4.err; exit 1; }
grep -A42 "attrib\]" gpurun_out/sdt_attrib_r4.err | head -45; cat gpurun_out/sdt_attrib_r4.json
(cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/sdt_prof_r4 -o sdt -- python3 $GRAFT_REPO_ROOT/bench/sd_bench.py --mode train --steps 4 --warmup 2 > $GRAFT_REPO_ROOT/gpurun_out/sdt_prof_r4.log 2>&1) || { echo "train prof failed"; tail -5 gpurun_out/sdt_prof_r4.log; exit 1; }
(cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/sdi_prof_r4 -o sdi -- python3 $GRAFT_REPO_ROOT/bench/sd_bench.py --mode infer --steps 2 --warmup 1 > $GRAFT_REPO_ROOT/gpurun_out/sdi_prof_r4.log 2>&1) || { echo "infer prof failed"; tail -5 gpurun_out/sdi_prof_r4.log; exit 1; }
for arm in 1 0; do
  KCA_SD_NARROW_TRAIN=$arm timeout -k 10 300 python -u bench/sd_bench.py --mode train --steps 8 --warmup 3 > gpurun_out/sdt_narrow$arm.json 2>/dev/null || exit 1
  echo "narrow_train=$arm $(cat gpurun_out/sdt_narrow$arm.json)"
  KCA_VAE_FLASH=$arm timeout -k 10 300 python -u bench/sd_bench.py --mode infer --steps 3 --warmup 1 > gpurun_out/sdi_vae$arm.json 2>/dev/null || exit 1
  echo "vae_flash=$arm $(cat gpurun_out/sdi_vae$arm.json)"
done
