"""SD UNet inference fusions on MI355X: the concat GroupNorm (no concatenated copy for the
norm, the upsampler's sub-pixel phase layout read in place) against cat + GroupNorm, the
im2col + GEMM phase upsampler (csrc/kernels/sd_upsample.hip) against nearest-x2 + conv3x3 in fp32,
and the fused UNet (phase upsamplers, concat GroupNorm, batched time projections) against the plain
path."""
import pytest
import torch
import torch.nn.functional as F

from kubernetes_cloud_amd.ops import _lib
from kubernetes_cloud_amd.ops.norms import group_norm, group_norm_cat, phase_to_dense

pytestmark = pytest.mark.gpu
DEV = "cuda"
CL = torch.channels_last


def _cl(*shape):
    return torch.randn(*shape, device=DEV, dtype=torch.bfloat16).contiguous(memory_format=CL)


@pytest.mark.parametrize("phase", [False, True])
@pytest.mark.parametrize("C1,C2,S", [(1280, 1280, 8), (640, 320, 16), (320, 320, 32)])
def test_group_norm_cat_matches_cat_then_norm(phase, C1, C2, S):
    torch.manual_seed(C1 + C2 + S)
    N, G = 2, 32
    x2 = _cl(N, C2, S, S)
    x1 = _cl(N, 4 * C1, S // 2 + 1, S // 2 + 1) if phase else _cl(N, C1, S, S)
    badd = torch.randn(C1, device=DEV, dtype=torch.bfloat16)
    w = torch.randn(C1 + C2, device=DEV, dtype=torch.bfloat16)
    b = torch.randn(C1 + C2, device=DEV, dtype=torch.bfloat16)
    with torch.no_grad():
        y, raw = group_norm_cat(x1, x2, G, w, b, 1e-5, silu=True, phase=phase, x1_add=badd)
        d1 = phase_to_dense(x1, (S, S)) if phase else x1
        cat = torch.cat([d1.float() + badd.float()[None, :, None, None], x2.float()], 1)
        ref = F.silu(F.group_norm(cat, G, w.float(), b.float(), 1e-5))
    assert _lib.has("kca_groupnorm_nhwc_cat_fwd")
    assert y.is_contiguous(memory_format=CL) and raw.is_contiguous(memory_format=CL)
    assert (raw.float() - cat).abs().max().item() <= 0.02 * cat.abs().max().item()
    assert (y.float() - ref).abs().max().item() < 0.05


def test_unet_phase_upsampler_and_fused_upblocks_match_plain(monkeypatch):
    from kubernetes_cloud_amd.models import unet
    from kubernetes_cloud_amd.models.unet import UNet2DConditionModel, UNetConfig, to_channels_last
    torch.manual_seed(0)
    cfg = UNetConfig(block_out_channels=(64, 128, 128, 128), cross_attention_dim=64, sample_size=32)
    m = to_channels_last(UNet2DConditionModel(cfg).to(DEV).bfloat16().eval())
    x = torch.randn(2, cfg.in_channels, 32, 32, device=DEV, dtype=torch.bfloat16)
    ctx = torch.randn(2, 8, cfg.cross_attention_dim, device=DEV, dtype=torch.bfloat16)
    with torch.no_grad():
        fused = m(x, 10, ctx)
        for flag in ("_PHASE_UP", "_CAT_GN", "_TEMB_BATCH"):
            monkeypatch.setattr(unet, flag, False)
        plain = m(x, 10, ctx)
    err = (fused.float() - plain.float()).abs().max().item()
    assert err < 0.03 * plain.float().abs().max().item() + 1e-3, err


@pytest.mark.parametrize("N,C,S", [(2, 64, 8), (3, 320, 16), (2, 1280, 4)])
def test_phase_gemm_upsampler_matches_fp32_reference(N, C, S):
    from kubernetes_cloud_amd.ops import upsample as up
    torch.manual_seed(N * C + S)
    x = _cl(N, C, S, S)
    w = (torch.randn(C, C, 3, 3, device=DEV) * (9 * C) ** -0.5).bfloat16()
    bias = torch.randn(C, device=DEV, dtype=torch.bfloat16)
    with torch.no_grad():
        a = up.im2col2x2(x)
        ref_a = up.im2col2x2(x.float())  # torch reference path (CPU/fp32 branch of the op)
        assert a.shape == ref_a.shape and torch.equal(a.float(), ref_a)
        t = up.upsample_conv_phase(x, up.phase_gemm_weights(w))
        dense = up.phase_to_dense(t, (2 * S, 2 * S), bias)
        ref = F.conv2d(F.interpolate(x.float(), scale_factor=2.0, mode="nearest"), w.float(), bias.float(), padding=1)
    assert _lib.has("kca_im2col2x2_nhwc") and _lib.has("kca_phase_to_dense_nhwc")
    assert dense.is_contiguous(memory_format=CL) and dense.shape == ref.shape
    err = (dense.float() - ref).abs().max().item()
    assert err < 0.03 * ref.abs().max().item(), err


def test_native_upsample2x_matches_interpolate():
    from kubernetes_cloud_amd.ops.upsample import upsample_nearest2x
    x = _cl(2, 96, 7, 5)
    with torch.no_grad():
        y = upsample_nearest2x(x)
    assert y.is_contiguous(memory_format=CL)
    assert torch.equal(y, F.interpolate(x, scale_factor=2.0, mode="nearest"))


def test_vae_decoder_phase_upsampler_matches_plain(monkeypatch):
    from kubernetes_cloud_amd.models import unet
    from kubernetes_cloud_amd.models.unet import to_channels_last
    from kubernetes_cloud_amd.models.vae import AutoencoderKL, VAEConfig
    torch.manual_seed(1)
    cfg = VAEConfig(block_out_channels=(64, 64, 128, 128))
    vae = to_channels_last(AutoencoderKL(cfg).to(DEV).bfloat16().eval())
    z = torch.randn(1, cfg.latent_channels, 16, 16, device=DEV, dtype=torch.bfloat16)
    with torch.no_grad():
        fused = vae.decode(z)
        monkeypatch.setattr(unet, "_PHASE_UP", False)
        plain = vae.decode(z)
    fused = fused.sample if hasattr(fused, "sample") else fused
    plain = plain.sample if hasattr(plain, "sample") else plain
    err = (fused.float() - plain.float()).abs().max().item()
    assert err < 0.03 * plain.float().abs().max().item() + 1e-3, err


def test_unet_graph_ctx_kv_cache_tracks_context():
    """sd_pipeline.UNetGraph projects the text K/V once per context tensor (CtxKV): replays with the
    same ctx reuse them, a new ctx recomputes them, and both match the eager UNet."""
    from kubernetes_cloud_amd.models.sd_pipeline import UNetGraph
    from kubernetes_cloud_amd.models.unet import UNet2DConditionModel, UNetConfig, to_channels_last
    torch.manual_seed(0)
    cfg = UNetConfig(block_out_channels=(64, 128, 128, 128), cross_attention_dim=64, sample_size=32)
    m = to_channels_last(UNet2DConditionModel(cfg).to(DEV).bfloat16().eval())
    g = UNetGraph(m)
    assert g.ctx_kv
    x = torch.randn(2, cfg.in_channels, 32, 32, device=DEV, dtype=torch.bfloat16)
    t = torch.full((2,), 10.0, device=DEV)
    c1 = torch.randn(2, 8, cfg.cross_attention_dim, device=DEV, dtype=torch.bfloat16)
    c2 = torch.randn(2, 8, cfg.cross_attention_dim, device=DEV, dtype=torch.bfloat16)
    with torch.no_grad():
        outs = []
        for c in (c1, c1, c2, c2, c1):
            outs.append(g(x, t, c).clone())
        e1, e2 = m(x, t, c1), m(x, t, c2)
    for o, e in zip(outs, (e1, e1, e2, e2, e1)):
        err = (o.float() - e.float()).abs().max().item()
        assert err < 0.02 * e.float().abs().max().item() + 1e-3, err


def test_unet_training_fusions_match_plain_grads(monkeypatch):
    """Training fusions (models/unet.py): conv biases folded into the time-embedding add and the
    residual add (ops.add_bias_nhwc_train, bias grads by column sums) and the padded heads from one
    fused QKV GEMM. Both bf16 paths are compared with an fp32 copy of the model (PyTorch reference
    ops): per parameter, the fused path's gradient error is within the plain path's bf16 noise."""
    import copy
    from kubernetes_cloud_amd.models import unet
    from kubernetes_cloud_amd.models.unet import UNet2DConditionModel, UNetConfig, to_channels_last
    torch.manual_seed(0)
    cfg = UNetConfig(block_out_channels=(320, 640, 640, 640), cross_attention_dim=64, sample_size=32)
    base = UNet2DConditionModel(cfg).to(DEV).train()
    m = to_channels_last(copy.deepcopy(base).bfloat16())
    ref = to_channels_last(base.float())
    x = torch.randn(2, cfg.in_channels, 32, 32, device=DEV).contiguous(memory_format=CL)
    ctx = torch.randn(2, 8, cfg.cross_attention_dim, device=DEV)
    tgt = torch.randn(2, cfg.out_channels, 32, 32, device=DEV, dtype=torch.float32)

    def run(model, dt):
        model.zero_grad(set_to_none=True)
        loss = F.mse_loss(model(x.to(dt), 10, ctx.to(dt)).float(), tgt)
        loss.backward()
        return loss.item(), {n: p.grad.float().clone() for n, p in model.named_parameters() if p.grad is not None}

    l1, g1 = run(m, torch.bfloat16)
    monkeypatch.setattr(unet, "_FOLD_BIAS_TRAIN", False)
    monkeypatch.setattr(unet, "_FUSED_QKV_TRAIN", False)
    l0, g0 = run(m, torch.bfloat16)
    lr, gr = run(ref, torch.float32)
    assert abs(l1 - lr) < 1e-2 * abs(lr) + 1e-4, (l1, l0, lr)
    assert set(g1) == set(g0) == set(gr)

    def rel(a, b):
        return ((a - b).norm() / (b.norm() + 1e-12)).item()
    bad = [(n, rel(g1[n], gr[n]), rel(g0[n], gr[n])) for n in gr
           if rel(g1[n], gr[n]) > max(2.0 * rel(g0[n], gr[n]), 0.03)]
    assert not bad, bad[:5]


@pytest.mark.parametrize("N,C,S,bias", [(2, 64, 8, True), (2, 320, 16, False), (1, 1280, 4, True)])
def test_phase_upsampler_training_grads_match_fp32(N, C, S, bias):
    """ops/upsample.py upsample_conv_train (im2col + GEMM + scatter, kca_dense_to_phase / col2im
    backward) against nearest-x2 + conv3x3 in fp32: output, dx, dW, db."""
    from kubernetes_cloud_amd.ops.upsample import upsample_conv_train
    torch.manual_seed(N + C + S)
    x = _cl(N, C, S, S).requires_grad_()
    w = ((torch.randn(C, C, 3, 3, device=DEV) * (9 * C) ** -0.5).bfloat16()
         .contiguous(memory_format=CL).requires_grad_())
    b = torch.randn(C, device=DEV, dtype=torch.bfloat16).requires_grad_() if bias else None
    g = torch.randn(N, C, 2 * S, 2 * S, device=DEV, dtype=torch.bfloat16).contiguous(memory_format=CL)
    y = upsample_conv_train(x, w, b)
    y.backward(g)
    xf, wf = x.detach().float().requires_grad_(), w.detach().float().requires_grad_()
    bf = b.detach().float().requires_grad_() if bias else None
    yf = F.conv2d(F.interpolate(xf, scale_factor=2.0, mode="nearest"), wf, bf, padding=1)
    yf.backward(g.float())
    assert _rel(y, yf) < 1e-2 and _rel(x.grad, xf.grad) < 2e-2 and _rel(w.grad, wf.grad) < 2e-2
    if bias:
        assert _rel(b.grad, bf.grad) < 1e-2


def _rel(a, b):
    a, b = a.float(), b.float()
    return ((a - b).norm() / (b.norm() + 1e-12)).item()


def test_unet_inference_caches_follow_native_optimizer_steps():
    """kca_adamw updates the bf16 parameters in place (no _version bump): the folded-bias,
    phase-GEMM, time-projection and context-K/V caches must still follow the new weights
    (TrainEngine._refresh_derived -> invalidate_weight_caches), e.g. DreamBooth's image logging."""
    import copy

    from kubernetes_cloud_amd.models.unet import UNet2DConditionModel, UNetConfig, to_channels_last
    from kubernetes_cloud_amd.train.engine import TrainEngine
    torch.manual_seed(0)
    cfg = UNetConfig(block_out_channels=(64, 128, 128, 128), cross_attention_dim=64, sample_size=32)
    m = to_channels_last(UNet2DConditionModel(cfg).to(DEV).bfloat16())
    x = torch.randn(2, cfg.in_channels, 32, 32, device=DEV, dtype=torch.bfloat16)
    ctx = torch.randn(2, 8, cfg.cross_attention_dim, device=DEV, dtype=torch.bfloat16)
    eng = TrainEngine(m, lr=1e-2, zero_stage=0)
    m.eval()
    with torch.no_grad():
        m(x, 10, ctx)  # populate every cache
        m.ctx_kv(ctx)
    m.train()
    eng.train_batch([x], lambda b: m(b, 10, ctx).float().pow(2).mean())
    m.eval()
    with torch.no_grad():
        got = m(x, 10, ctx)
        fresh = copy.deepcopy(m)  # same weights, no caches
        for mod in fresh.modules():
            for a in ("_fb_cache", "_phase_cache", "_temb_cache", "_ctxkv_cache"):
                if hasattr(mod, a):
                    delattr(mod, a)
        ref = fresh(x, 10, ctx)
    # a stale cache after an lr 1e-2 Adam step is off by O(1); a rebuilt one by bf16 rounding (the
    # caches fold weights in fp32 and round once: 1 ulp at the output's max, 2^-6 at 3.5)
    err = (got.float() - ref.float()).abs().max().item()
    assert _rel(got, ref) < 5e-3 and err <= 1e-2 * ref.float().abs().max().item(), (err, _rel(got, ref))


def test_vae_encoder_conv_in_bias_fold_matches_plain():
    """Inference VAE encode: conv_in's bias carried by the first ResNet block (GroupNorm add +
    residual add) equals the plain biased convolution; the channels-last Downsample2D pad kernel too."""
    from kubernetes_cloud_amd.models.unet import to_channels_last
    from kubernetes_cloud_amd.models.vae import AutoencoderKL, VAEConfig
    torch.manual_seed(2)
    vae = to_channels_last(AutoencoderKL(VAEConfig(block_out_channels=(64, 128, 128, 128))).to(DEV).bfloat16().eval())
    for p_ in vae.parameters():
        if p_.dim() == 1:
            torch.nn.init.normal_(p_, std=0.1)
    x = torch.randn(2, 3, 64, 64, device=DEV).bfloat16().contiguous(memory_format=torch.channels_last)
    with torch.no_grad():
        got = vae.encode_moments(x)
    with torch.enable_grad():  # the unfolded path (and F.pad in the downsamplers)
        ref = vae.encode_moments(x).detach()
    assert _rel(got, ref) < 1e-2


@pytest.mark.parametrize("tokens", [4096, 65536])
def test_linear_residual_train_grads_match_reference(tokens):
    """Training res + x W^T + b in one GEMM epilogue (ops.linear_residual_train): the output and the
    x / W / b / res gradients match the two-pass autograd form in fp32."""
    from kubernetes_cloud_amd.ops.linear import linear_residual_train
    torch.manual_seed(4)
    K, N = 640, 320
    x = (torch.randn(tokens, K, device=DEV) * 0.5).bfloat16().requires_grad_(True)
    w = (torch.randn(N, K, device=DEV) / K ** 0.5).bfloat16().requires_grad_(True)
    b = torch.randn(N, device=DEV).bfloat16().requires_grad_(True)
    r = torch.randn(tokens, N, device=DEV).bfloat16().requires_grad_(True)
    y = linear_residual_train(x, w, b, r)
    g = torch.randn_like(y)
    y.backward(g)
    xf, wf, bf, rf = (t.detach().float().requires_grad_(True) for t in (x, w, b, r))
    yf = rf + xf @ wf.t() + bf
    yf.backward(g.float())
    assert _rel(y, yf) < 1e-2
    for got, ref in ((x.grad, xf.grad), (w.grad, wf.grad), (b.grad, bf.grad), (r.grad, rf.grad)):
        assert _rel(got, ref) < 2e-2
