"""GPU debug: runner.prefill logits vs full forward, per config."""
import sys
import torch
sys.path.insert(0, ".")
from kubernetes_cloud_amd.engine.runner import ModelRunner
from kubernetes_cloud_amd.models.causal_lm import build_model
from kubernetes_cloud_amd.models.config import PRESETS_HF, LMConfig
from kubernetes_cloud_amd import ops

dev = torch.device("cuda", 0)
for name, over in (("gpt-j-6b", dict(n_embd=1024, n_layer=2, n_head=4, rotary_dim=64, n_positions=512)),
                   ("gpt-j-6b", dict(n_embd=1024, n_layer=1, n_head=8, rotary_dim=64, n_positions=512)),
                   ("pythia-2.8b", dict(hidden_size=1024, num_hidden_layers=2, num_attention_heads=8,
                                        intermediate_size=4096, max_position_embeddings=512))):
    cfg = dict(PRESETS_HF[name]); cfg.update(over)
    m = build_model(LMConfig.from_hf(cfg), device=dev, dtype=torch.bfloat16, seed=0).eval()
    r = ModelRunner(m, max_slots=4, max_len=256, use_graphs=False)
    for n, T in ((1, 5), (2, 5), (1, 33)):
        ids = torch.randint(0, 1000, (n, T), device=dev)
        with torch.no_grad():
            a = r.prefill(ids, list(range(n))).float()
            b = m(ids)[:, -1].float()
        print(name, over.get("n_head", over.get("num_attention_heads")), n, T, "maxdiff", float((a - b).abs().max()),
              "argmax eq", bool((a.argmax(-1) == b.argmax(-1)).all()), flush=True)
    # rope on strided view vs reference
    D = m.cfg.head_dim; H = m.cfg.n_heads; rot = m.cfg.rotary_dim
    qkv = torch.randn(2, 5, 3, H, D, device=dev).to(torch.bfloat16)
    ref_q = ops.rotary_reference(qkv[:, :, 0].float(), rot, m.cfg.rotary_interleaved, m.cfg.rotary_base)
    q, k = qkv[:, :, 0], qkv[:, :, 1]
    ops.apply_rotary_(q, k, rot, 5, m.cfg.rotary_interleaved, m.cfg.rotary_base, max_pos=256)
    print("rope diff", float((q.float() - ref_q).abs().max()), flush=True)
