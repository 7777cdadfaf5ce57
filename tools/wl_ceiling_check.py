import json, os, sys, torch
sys.path.insert(0, os.getcwd())
sys.path.insert(0, os.path.join(os.getcwd(), "bench"))
import weight_load_bench as wl
d = os.environ.get("TMPDIR", "/tmp")
out = wl.run_weight_load("gpt-j-6b", d, threads=8, sources=("cold",))
torch.cuda.empty_cache()
out += wl.run_weight_load("bloom-176b", d, threads=8, sources=("cold",), tp=8, layers=10)
for r in out:
    print(json.dumps({k: r[k] for k in ("model", "gbps", "storage_gbps", "of_storage", "read_path")}), flush=True)
