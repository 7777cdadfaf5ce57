"""Sampler latency (kca_sample_logits) at GPT-J's vocabulary, batch 1 and 32: greedy, top-k 10 (the
FasterTransformer request), top-k 50, top-k 50 + top-p 0.95 (the finetuner / HF defaults), top-p only.
Rows with 1 <= top_k <= 64 or greedy run on the multi-workgroup sampler; KCA_SAMPLE_MWG=0 puts them
on the one-workgroup register kernel (A/B). Kernel times: rocprofv3 --kernel-trace --stats."""
import sys, time, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from kubernetes_cloud_amd.ops import decode as dops

dev = torch.device("cuda", 0)
V = 50400
for B in (1, 32):
    logits = (torch.randn(B, V, device=dev) * 4).to(torch.bfloat16)
    for name, (t, k, p) in {"greedy": (0.0, 0, 1.0), "topk10": (1.0, 10, 1.0), "topk50": (1.0, 50, 1.0),
                          "topk50_topp0.95": (1.0, 50, 0.95), "topp0.95": (1.0, 0, 0.95)}.items():
        f = lambda v, dt: torch.full((B,), v, dtype=dt, device=dev)  # noqa: E731
        kw = dict(temperature=f(t, torch.float32), top_k=f(k, torch.int32), top_p=f(p, torch.float32),
                  rep_penalty=f(1.0, torch.float32), seeds=torch.arange(B, device=dev),
                  mwg_complete=dops.mwg_complete_rows([t] * B, [k] * B))  # as the decode engine passes it
        for _ in range(5):
            dops.sample_logits(logits, **kw)
        torch.cuda.synchronize()
        n = 200
        t0 = time.perf_counter()
        for _ in range(n):
            dops.sample_logits(logits, **kw)
        torch.cuda.synchronize()
        print(f"B={B} {name}: {(time.perf_counter() - t0) / n * 1e6:.1f} us/call (host-launched, incl. launch)")
