"""Sliding-window (GPT-Neo local layers) and per-key-hole masks in the HIP
attention kernels (csrc/kernels/attention.hip, decode.hip) against the fp32
PyTorch reference -- forward and backward -- and the GPT-Neo engine on the
GPU with HIP graphs against full recompute."""
import pytest
import torch

from kubernetes_cloud_amd import ops
from kubernetes_cloud_amd.ops import decode as dops
from kubernetes_cloud_amd.ops.attention import attention_reference

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _rel(a, b):
    a, b = a.float(), b.float()
    return ((a - b).norm() / (b.norm() + 1e-12)).item()


def _fwd_bwd(q, k, v, **kw):
    o = ops.flash_attention(q, k, v, causal=True, **kw)
    g = torch.randn_like(o)
    dq, dk, dv = torch.autograd.grad(o, (q, k, v), g)
    qr, kr, vr = (t.detach().float().requires_grad_() for t in (q, k, v))
    ref_kw = dict(kw)
    ref_kw.pop("scale", None)
    orf, _ = attention_reference(qr, kr, vr, True, kw.get("scale"), kw.get("kv_len"), None, kw.get("window", 0))
    drq, drk, drv = torch.autograd.grad(orf, (qr, kr, vr), g.float())
    return (o, dq, dk, dv), (orf, drq, drk, drv)


@pytest.mark.parametrize("D,S,W", [(64, 700, 256), (128, 1024, 256), (64, 512, 100), (256, 512, 64)])
def test_window_fwd_bwd(D, S, W):
    torch.manual_seed(D + S + W)
    B, H = 2, 4
    q, k, v = (torch.randn(B, S, H, D, device=DEV, dtype=torch.bfloat16).requires_grad_() for _ in range(3))
    got, ref = _fwd_bwd(q, k, v, window=W, scale=1.0 if D == 64 else None)
    for a, b, name in zip(got, ref, ("o", "dq", "dk", "dv")):
        assert _rel(a, b) < 2e-2, (name, _rel(a, b))


@pytest.mark.parametrize("D", [64, 128, 256])
def test_key_holes_fwd_bwd(D):
    """Interior EOS separators (pad == eos last context): a bool per-key mask
    with holes, through the kernels as a bitmap (no fp32 reference path)."""
    torch.manual_seed(D)
    B, S, H = 2, 384, 4
    q, k, v = (torch.randn(B, S, H, D, device=DEV, dtype=torch.bfloat16).requires_grad_() for _ in range(3))
    mask = torch.ones(B, S, dtype=torch.bool)
    mask[0, 100:104] = False
    mask[0, 250] = False
    mask[1, 31:33] = False
    mask[1, 300:] = False
    got, ref = _fwd_bwd(q, k, v, kv_len=mask)
    for a, b, name in zip(got, ref, ("o", "dq", "dk", "dv")):  # every row sees key 0: none fully masked
        assert _rel(a, b) < 2e-2, name
    assert float(got[2][1, 300:].abs().max()) == 0.0  # masked keys get no gradient


def test_mask_bitmap_packing():
    from kubernetes_cloud_amd.ops.attention import pack_key_mask
    m = torch.rand(3, 77) > 0.3
    w = pack_key_mask(m)
    assert w.shape == (3, 3) and w.dtype == torch.int32
    bits = ((w.to(torch.int64) & 0xFFFFFFFF)[:, :, None] >> torch.arange(32)) & 1
    assert torch.equal(bits.view(3, 96)[:, :77].bool(), m)


@pytest.mark.parametrize("W,L", [(256, 700), (64, 300), (512, 200)])
def test_decode_window(W, L):
    torch.manual_seed(W)
    B, H, D, slots_n = 3, 4, 64, 4
    kc = torch.randn(slots_n, H, 1024, D, device=DEV, dtype=torch.bfloat16)
    vc = torch.randn_like(kc)
    q = torch.randn(B, H * D, device=DEV, dtype=torch.bfloat16)
    slots = torch.tensor([2, 0, 3], device=DEV, dtype=torch.int32)
    lens = torch.tensor([L, L // 2 + 1, 17], device=DEV, dtype=torch.int32)
    for chunk in (64, 256, 0):
        o = dops.decode_attention(q, kc, vc, slots, lens, H, L, chunk=chunk, window=W)
        r = dops.decode_attention_reference(q.cpu(), kc.cpu(), vc.cpu(), slots.cpu(), lens.cpu(), H,
                                            1.0 / D ** 0.5, window=W)
        assert _rel(o.cpu(), r) < 1e-2, chunk


def test_gpt_neo_engine_graphs_and_training_on_kernels():
    """GPT-Neo (global + local layers): the engine's HIP-graph decode equals
    greedy recompute, and a training step runs with no fp32 softmax on the GPU."""
    from kubernetes_cloud_amd.engine.llm_engine import LLMEngine, SamplingParams
    from kubernetes_cloud_amd.models.causal_lm import build_model
    from kubernetes_cloud_amd.models.config import LMConfig
    cfg = {"model_type": "gpt_neo", "vocab_size": 1000, "hidden_size": 512, "num_layers": 4, "num_heads": 8,
           "attention_types": [[["global", "local"], 2]], "window_size": 64, "max_position_embeddings": 512}
    m = build_model(LMConfig.from_hf(cfg), device=DEV, dtype=torch.bfloat16, seed=0)
    eng = LLMEngine(m, max_slots=4, max_len=400)
    assert eng.runner.use_graphs
    g = torch.Generator().manual_seed(0)
    prompt = [int(x) for x in torch.randint(0, 1000, (150,), generator=g)]
    out = eng.generate([prompt], SamplingParams(max_new_tokens=24, do_sample=False))[0].output
    ids = list(prompt)
    for _ in range(24):
        with torch.no_grad():
            row = m(torch.tensor([ids], device=DEV))[0, -1].float()
        ids.append(int(row.argmax()))
    ref = ids[len(prompt):]
    i = next((j for j, (a, b) in enumerate(zip(out, ref)) if a != b), None)
    if i is not None:
        with torch.no_grad():
            row = m(torch.tensor([prompt + ref[:i]], device=DEV))[0, -1].float()
        top2 = row.topk(2).values
        assert float(top2[0] - top2[1]) < 0.1, i
    # training step: profile for any aten softmax kernel (the old fp32 local-attention path)
    m.train()
    x = torch.randint(0, 1000, (2, 256), device=DEV)
    with torch.profiler.profile(activities=[torch.profiler.ProfilerActivity.CUDA]) as prof:
        loss = m(x, labels=x)
        loss.backward()
        torch.cuda.synchronize()
    names = [e.name for e in prof.events()]
    assert not any("softmax" in n.lower() for n in names), [n for n in names if "softmax" in n.lower()][:5]
    assert any("attn" in n for n in names)


def test_rowsum_column_variant_matches_reference():
    """SD-1.5 padded heads (40 -> 64): V column 40 = 1 lets the D=64 kernel take
    the softmax row sums from O; output equals the fp32 reference on the real
    40 dims and is 1.0 in column 40."""
    torch.manual_seed(7)
    B, S, H = 2, 4096, 8
    q, k, v = (torch.zeros(B, S, H, 64, device=DEV, dtype=torch.bfloat16) for _ in range(3))
    for t in (q, k, v):
        t[..., :40] = torch.randn(B, S, H, 40, device=DEV).bfloat16()
    v[..., 40] = 1.0
    with torch.no_grad():
        o = ops.flash_attention(q, k, v, causal=False, scale=40 ** -0.5, rowsum_col=40)
        o_plain = ops.flash_attention(q, k, v, causal=False, scale=40 ** -0.5)
    ref, _ = attention_reference(q[..., :40], k[..., :40], v[..., :40], False, 40 ** -0.5)
    assert _rel(o[..., :40], ref) < 1e-2
    assert _rel(o_plain[..., :40], ref) < 1e-2
    assert float((o[..., 40].float() - 1).abs().max()) < 2e-2


def test_unet_padded_attention_rowsum_matches_unpadded():
    from kubernetes_cloud_amd.models.unet import Attention
    torch.manual_seed(3)
    att = Attention(320, 8, 40).to(DEV).bfloat16().eval()
    for p_ in att.parameters():
        torch.nn.init.normal_(p_, std=0.05)
    x = torch.randn(2, 4096, 320, device=DEV, dtype=torch.bfloat16)
    with torch.no_grad():
        fast = att(x)  # padded heads + rowsum column
        q, k_, v = att.to_q(x), att.to_k(x), att.to_v(x)
        ref, _ = attention_reference(q.view(2, 4096, 8, 40), k_.view(2, 4096, 8, 40), v.view(2, 4096, 8, 40),
                                     False, 40 ** -0.5)
        ref = att.to_out[0](ref.reshape(2, 4096, 320).to(torch.bfloat16))
    assert _rel(fast, ref) < 2e-2


@pytest.mark.parametrize("rowsum", [False, True])
def test_narrow_48_storage_matches_reference(rowsum):
    """SD-1.5 inference heads stored 48 wide (40 real + 8 zero) in a packed QKV
    tensor, staged into the D=64 LDS image (StagerNarrow): equals the fp32
    reference on the 40 real dims, and the narrow tiled kernel is the one that ran."""
    torch.manual_seed(11)
    B, S, H = 2, 2048, 8
    qkv = torch.zeros(B, S, 3, H, 48, device=DEV, dtype=torch.bfloat16)
    qkv[..., :40] = torch.randn(B, S, 3, H, 40, device=DEV).bfloat16()
    if rowsum:
        qkv[:, :, 2, :, 40] = 1.0
    q, k, v = qkv[:, :, 0], qkv[:, :, 1], qkv[:, :, 2]
    with torch.no_grad(), torch.profiler.profile(activities=[torch.profiler.ProfilerActivity.CUDA]) as prof:
        o = ops.flash_attention(q, k, v, causal=False, scale=40 ** -0.5, rowsum_col=40 if rowsum else -1)
        torch.cuda.synchronize()
    ref, _ = attention_reference(q[..., :40], k[..., :40], v[..., :40], False, 40 ** -0.5)
    assert o.shape == (B, S, H, 48)
    assert _rel(o[..., :40], ref) < 1e-2
    if rowsum:
        assert float((o[..., 40].float() - 1).abs().max()) < 2e-2
    else:
        assert float(o[..., 40:].float().abs().max()) == 0.0
    names = [e.name for e in prof.events()]
    assert any("attn_fwd_tiled" in n and "48" in n for n in names), sorted(set(names))[:8]


def test_unet_inference_heads_are_48_wide():
    from kubernetes_cloud_amd.models import unet
    assert unet.padded_head_dim(40, infer=True) == 48
    assert unet.padded_head_dim(40) == 48  # fwd + bwd narrow kernels
    assert unet.padded_head_dim(80, infer=True) == 96


def test_narrow_48_backward_matches_fp32_reference():
    """Training heads stored 48 wide (40 real + 8 zero) in ONE fused QKV buffer
    (models/unet.py, ops.qkv_rope_attention): the DS = 48 dQ and dK/dV kernels
    (attention_tiled.hip, D = 64 images, pad chunks zeroed in LDS) give the fp32
    reference gradients on the 40 real dims, zeros on the pad, and are the ones that ran."""
    torch.manual_seed(17)
    B, S, H = 2, 1024, 8
    base = torch.zeros(B, S, 3, H, 48, device=DEV)
    base[..., :40] = torch.randn(B, S, 3, H, 40, device=DEV)
    qkv = base.bfloat16().view(B, S, 3 * H * 48).requires_grad_(True)
    g = torch.randn(B, S, H, 48, device=DEV).bfloat16()
    g[..., 40:] = 0
    with torch.profiler.profile(activities=[torch.profiler.ProfilerActivity.CUDA]) as prof:
        o = ops.qkv_rope_attention(qkv, H, 48, 0, False, causal=False, scale=40 ** -0.5)
        o.backward(g.view(B, S, H * 48))
        torch.cuda.synchronize()
    ref_in = qkv.detach().float().view(B, S, 3, H, 48)[..., :40].clone().requires_grad_(True)
    ro, _ = attention_reference(ref_in[:, :, 0], ref_in[:, :, 1], ref_in[:, :, 2], False, 40 ** -0.5)
    ro.backward(g[..., :40].float())
    gq = qkv.grad.view(B, S, 3, H, 48)
    assert float(gq[..., 40:].float().abs().max()) == 0.0
    for i in range(3):
        assert _rel(gq[:, :, i, :, :40], ref_in.grad[:, :, i]) < 2e-2, i
    names = [e.name for e in prof.events()]
    for kern in ("attn_bwd_dq_tiled", "attn_bwd_dkdv_tiled"):
        assert any(kern in n and "48" in n for n in names), (kern, sorted(set(names))[:12])


def test_narrow_48_max_column_matches_reference():
    """attention_tiled.hip MC: K pre-scaled by s*log2(e) with pad column 40 = 1, scale = ln 2, V column
    40 = 1 (row sums): the S MFMAs carry the softmax offset; equals the fp32 reference at scale s."""
    import math
    torch.manual_seed(13)
    B, S, H = 2, 2048, 8
    s = 40 ** -0.5
    qkv = torch.zeros(B, S, 3, H, 48, device=DEV, dtype=torch.bfloat16)
    qkv[..., :40] = (torch.randn(B, S, 3, H, 40, device=DEV) * 1.5).bfloat16()
    ref, lse_ref = attention_reference(qkv[:, :, 0, :, :40], qkv[:, :, 1, :, :40], qkv[:, :, 2, :, :40], False, s)
    qkv[:, :, 1, :, :40] = (qkv[:, :, 1, :, :40].float() * s * math.log2(math.e)).bfloat16()
    qkv[:, :, 1, :, 40] = 1.0
    qkv[:, :, 2, :, 40] = 1.0
    q, k, v = qkv[:, :, 0], qkv[:, :, 1], qkv[:, :, 2]
    with torch.no_grad(), torch.profiler.profile(activities=[torch.profiler.ProfilerActivity.CUDA]) as prof:
        o = ops.flash_attention(q, k, v, causal=False, scale=math.log(2.0), rowsum_col=40, max_col=40)
        torch.cuda.synchronize()
    assert _rel(o[..., :40], ref) < 1.5e-2
    assert float((o[..., 40].float() - 1).abs().max()) < 2e-2
    names = [e.name for e in prof.events()]
    assert any("attn_fwd_tiled" in n and "40, 48, 40" in n for n in names), sorted(set(names))[:8]


def test_unet_attention_max_column_matches_plain(monkeypatch):
    from kubernetes_cloud_amd.models import unet
    from kubernetes_cloud_amd.models.unet import Attention
    torch.manual_seed(5)
    att = Attention(320, 8, 40).to(DEV).bfloat16().eval()
    for p_ in att.parameters():
        torch.nn.init.normal_(p_, std=0.05)
    x = torch.randn(2, 4096, 320, device=DEV, dtype=torch.bfloat16)
    with torch.no_grad():
        fast = att(x)
        monkeypatch.setattr(unet, "_MAX_COL", False)
        plain = att(x)
    assert _rel(fast, plain) < 2e-2


def test_wide_head_512_flash_matches_reference():
    """The VAE mid-block's single 512-wide head on the 4-wave LDS-DMA flash kernel
    (attention_tiled.hip attn_fwd_w8_kernel<512, false, 4, 2>) against the fp32 reference,
    with no [B, S, S] score tensor or softmax kernel on the way."""
    from kubernetes_cloud_amd.ops.attention import wide_head_attention
    torch.manual_seed(19)
    B, S, C = 2, 1024, 512
    q, k, v = (torch.randn(B, S, C, device=DEV) * 0.5).bfloat16(), torch.randn(B, S, C, device=DEV).bfloat16(), \
        torch.randn(B, S, C, device=DEV).bfloat16()
    with torch.no_grad(), torch.profiler.profile(activities=[torch.profiler.ProfilerActivity.CUDA]) as prof:
        o = wide_head_attention(q, k, v, C ** -0.5)
        torch.cuda.synchronize()
    assert o is not None
    ref, _ = attention_reference(q[:, :, None], k[:, :, None], v[:, :, None], False, C ** -0.5)
    assert _rel(o, ref[:, :, 0]) < 1e-2
    names = [e.name for e in prof.events()]
    assert any("attn_fwd_w8_kernel" in n and "512" in n for n in names), sorted(set(names))[:8]
    assert not any("softmax" in n.lower() for n in names)


def test_vae_mid_attention_uses_wide_flash():
    from kubernetes_cloud_amd.models import vae as vae_mod
    torch.manual_seed(23)
    att = vae_mod.VAEAttention(512, 32).to(DEV).bfloat16().eval()
    x = torch.randn(2, 512, 32, 32, device=DEV).bfloat16()
    with torch.no_grad():
        fast = att(x)
        vae_mod._FLASH_WIDE = False
        try:
            slow = att(x)
        finally:
            vae_mod._FLASH_WIDE = True
    assert _rel(fast, slow) < 1e-2
