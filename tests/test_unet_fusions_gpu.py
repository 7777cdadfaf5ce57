"""SD UNet inference fusions on MI355X: the concat GroupNorm (no concatenated copy for the
norm, the upsampler's sub-pixel phase layout read in place) against cat + GroupNorm, and the
phase-conv upsampler + fused up-block against the plain UNet path."""
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
        monkeypatch.setattr(unet, "_FUSE_UP", False)
        plain = m(x, 10, ctx)
    err = (fused.float() - plain.float()).abs().max().item()
    assert err < 0.03 * plain.float().abs().max().item() + 1e-3, err
