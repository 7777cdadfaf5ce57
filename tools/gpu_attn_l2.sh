# L2 hit rate of the attention kernels at the GPT-J training shape (one PMC pass + trace).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/pmc_l2
mkdir -p $OUT
timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE -d $OUT/l2 -o l2 --output-format csv -- \
  python3 bench/kernel_pmc.py --cases attn_gptj --out $OUT/cases.json > $OUT/l2.log 2>&1 || exit 1
f=$(find $OUT/l2 -name "*counter_collection.csv" | head -1)
python3 - "$f" <<'PY'
import csv, sys, collections
acc = collections.defaultdict(lambda: collections.defaultdict(float))
for r in csv.DictReader(open(sys.argv[1])):
    acc[r["Kernel_Name"][:60]][r["Counter_Name"]] += float(r["Counter_Value"])
for k, v in acc.items():
    h, m = v.get("TCC_HIT_sum", 0), v.get("TCC_MISS_sum", 0)
    if h + m > 0:
        print(f"{k:60s} hit={h:.3g} miss={m:.3g} hit_rate={h / (h + m):.3f}")
PY
