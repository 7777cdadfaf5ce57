# round-4 batch 19: fresh GPT-J B=1 decode timeline (current fused layer kernels)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
bash tools/gpu_decode_timeline.sh || { tail -20 gpurun_out/dec_tl.log; exit 1; }
tail -3 gpurun_out/dec_tl.log
f=$(find gpurun_out/dec_tl -name '*kernel_trace.csv' | head -1)
echo "trace: $f"
python3 - "$f" <<'PY'
import csv, sys, collections
c = collections.Counter(r["Kernel_Name"].split("(")[0][:60] for r in csv.DictReader(open(sys.argv[1])))
for k, v in c.most_common(15): print(v, k)
PY
for sk in sample_kernel sample_reg_kernel sample_mwg_kernel; do
  python3 tools/timeline.py "$f" --step-kernel $sk --show 12 > gpurun_out/dec_tl_r4.txt 2>&1 && break
done
cat gpurun_out/dec_tl_r4.txt
