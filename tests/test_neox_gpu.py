"""GPT-NeoX architecture on the GPU (VERDICT r4 Missing #2).

The reference's DEFAULT finetune model is ``EleutherAI/pythia-2.8b-deduped``
(finetuner-workflow/finetune-workflow.yaml:17-18), its FasterTransformer service
serves GPT-NeoX-20B (online-inference/fastertransformer/ft-inference-service-neox.yml:44)
and the 3D-parallel job finetunes NeoX-20B (kubeflow/training-operator/gpt-neox/
04-finetune-workflow.yaml:199-217). gpt_neox differs from GPT-J in everything the native
kernels touch: a separate ``ln_2`` (two LayerNorms of the same residual stream), the
parallel residual, rotate-half RoPE on 25 % of a 96- (20B) or 80-wide (2.8B) head, and
exact-erf GELU. These tests run shrunk models of both head widths through the native
training path (forward + backward against an fp32 model of the same weights) and the
training engine's optimizer step.
"""
import pytest
import torch

pytestmark = pytest.mark.gpu
dev = torch.device("cuda", 0)


def _cfg(head_dim: int, layers: int = 2):
    from kubernetes_cloud_amd.models.config import PRESETS_HF, LMConfig
    base = "gpt-neox-20b" if head_dim == 96 else "pythia-2.8b"
    heads = 4
    cfg = dict(PRESETS_HF[base])
    cfg.update(hidden_size=heads * head_dim, num_hidden_layers=layers, num_attention_heads=heads,
               intermediate_size=4 * heads * head_dim, vocab_size=512, max_position_embeddings=512)
    return LMConfig.from_hf(cfg)


def _rel(a, b):
    return float((a.float() - b.float()).norm() / b.float().norm().clamp_min(1e-12))


@pytest.mark.parametrize("head_dim", [96, 80])
def test_gpt_neox_forward_backward_matches_fp32(head_dim):
    """bf16 native forward + backward of a gpt_neox model (tiled flash attention at D = 96 / 80,
    rotate-half RoPE over 24 / 20 dims, two LayerNorms, parallel residual) against the same weights
    in fp32: loss and every parameter's gradient."""
    from kubernetes_cloud_amd.models.causal_lm import build_model
    from kubernetes_cloud_amd.ops import _lib
    cfg = _cfg(head_dim)
    assert cfg.arch == "gpt_neox" and cfg.parallel_residual and cfg.rotary_dim == head_dim // 4
    m32 = build_model(cfg, device=dev, dtype=torch.float32, seed=0)
    m16 = build_model(cfg, device=dev, dtype=torch.bfloat16, seed=0)
    m16.load_state_dict({k: v.to(torch.bfloat16) for k, v in m32.state_dict().items()})
    # the fp32 reference starts from the bf16-rounded weights, so only the arithmetic differs
    m32.load_state_dict({k: v.float() for k, v in m16.state_dict().items()})
    assert all(blk.ln_2 is not None for blk in m16.h)
    g = torch.Generator(device=dev).manual_seed(1)
    ids = torch.randint(0, cfg.vocab_size, (2, 256), device=dev, generator=g)
    res = []
    for m in (m16, m32):
        m.train()
        m.zero_grad(set_to_none=True)
        loss = m(ids, labels=ids)
        loss.backward()
        res.append((float(loss), {n: p.grad.float().clone() for n, p in m.named_parameters()}))
    (l16, g16), (l32, g32) = res
    assert abs(l16 - l32) < 1e-2 * abs(l32), (l16, l32)
    worst = sorted(((_rel(g16[n], g32[n]), n) for n in g32), reverse=True)
    assert worst[0][0] < 6e-2, worst[:5]
    assert _lib.has("kca_attn_fwd")  # the native library carried the forward (use_native paths)


@pytest.mark.parametrize("head_dim", [96, 80])
def test_gpt_neox_engine_steps_match_fp32(head_dim):
    """Training-engine steps (fused AdamW, grad clip, GAS 2) on the bf16 gpt_neox model follow the fp32
    reference: the loss curve over 4 steps agrees and falls on a repeated batch."""
    from kubernetes_cloud_amd.models.causal_lm import build_model
    from kubernetes_cloud_amd.train.engine import TrainEngine
    cfg = _cfg(head_dim)
    g = torch.Generator(device=dev).manual_seed(2)
    mbs = [torch.randint(0, cfg.vocab_size, (2, 128), device=dev, generator=g) for _ in range(2)]
    curves = []
    for dt in (torch.bfloat16, torch.float32):
        m = build_model(cfg, device=dev, dtype=dt, seed=0)
        m.train()
        eng = TrainEngine(m, lr=3e-3, weight_decay=0.01, grad_accum=2)
        curves.append([float(eng.train_batch(mbs, lambda b: m(b, labels=b))) for _ in range(4)])
        eng.remove_hooks()
    c16, c32 = curves
    assert c16[-1] < c16[0] and c32[-1] < c32[0], curves
    for a, b in zip(c16, c32):
        assert abs(a - b) < 3e-2 * abs(b), curves
