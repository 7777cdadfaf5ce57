"""TrainEngine with / without optimizer offload on a tiny GPT-J: where do they diverge?"""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch
from kubernetes_cloud_amd.models.causal_lm import build_model
from kubernetes_cloud_amd.models.config import LMConfig, PRESETS_HF
from kubernetes_cloud_amd.train.engine import TrainEngine
from kubernetes_cloud_amd.train.optim import HostOffloadAdamW

DEV = "cuda"
cfg = dict(PRESETS_HF["gpt-j-6b"])
cfg.update(n_embd=256, n_layer=2, n_head=4, rotary_dim=32, vocab_size=1024)
torch.manual_seed(0)
ids = torch.randint(0, 1024, (2, 128), device=DEV)
snaps = {}
for off in (False, True):
    m = build_model(LMConfig.from_hf(cfg), device=DEV, dtype=torch.bfloat16, seed=0)
    HostOffloadAdamW.CHUNK = 1 << 16
    eng = TrainEngine(m, lr=1e-3, weight_decay=0.01, grad_accum=1, offload_optimizer=off)
    s = [eng.flat.float().clone()]
    for _ in range(3):
        loss = eng.train_batch([ids], lambda b: m(b, labels=b))
        torch.cuda.synchronize()
        s.append(eng.flat.float().clone())
        s.append(eng.grad.clone())
    snaps[off] = (s, eng)
a, b = snaps[False][0], snaps[True][0]
names = [(sl.name, sl.offset, sl.numel) for sl in snaps[False][1].slots]
for k, (x, y) in enumerate(zip(a, b)):
    d = (x - y).abs()
    bad = (d > 1e-2 * (x.abs().max() + 1e-6)).nonzero().flatten()
    where = [n for n, o, c in names if bad.numel() and o <= int(bad[0]) < o + c]
    print(k, "max", float(d.max()), "nbad", bad.numel(), "first", bad[:3].tolist(), where)
