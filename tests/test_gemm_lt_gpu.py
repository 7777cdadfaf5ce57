"""hipBLASLt GEMM with bias + residual epilogue (csrc/kernels/gemm_lt.hip, ops.linear_residual)
against an fp32 PyTorch reference, including the channels-last token view the SD UNet passes."""
import pytest
import torch

from kubernetes_cloud_amd.ops import _lib
from kubernetes_cloud_amd.ops.linear import linear_residual

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _ref(x, w, b, r):
    y = x.float() @ w.float().t()
    if b is not None:
        y = y + b.float()
    return r.float() + y.reshape(r.shape)


@pytest.mark.parametrize("M,N,K,bias", [(4096, 320, 1280, True), (1000, 640, 320, False), (256, 1280, 5120, True)])
def test_linear_residual_matches_fp32(M, N, K, bias):
    torch.manual_seed(M + N)
    x = torch.randn(M, K, device=DEV, dtype=torch.bfloat16)
    w = (torch.randn(N, K, device=DEV) * K ** -0.5).bfloat16()
    b = torch.randn(N, device=DEV, dtype=torch.bfloat16) if bias else None
    r = torch.randn(M, N, device=DEV, dtype=torch.bfloat16)
    with torch.no_grad():
        out = linear_residual(x, w, b, r)
        out2 = linear_residual(x, w, b, r)  # the tuned plan
    ref = _ref(x, w, b, r)
    assert out.shape == r.shape and out.dtype == torch.bfloat16
    for o in (out, out2):
        err = (o.float() - ref).abs().max().item()
        assert err < 0.05 * ref.abs().max().item(), err


def test_linear_residual_channels_last_view_and_graph():
    """res as the permuted NHWC view of a channels-last NCHW tensor; then captured in a HIP graph."""
    torch.manual_seed(0)
    B, C, H, W = 2, 320, 16, 16
    res = torch.randn(B, C, H, W, device=DEV, dtype=torch.bfloat16).contiguous(memory_format=torch.channels_last)
    t = torch.randn(B, H * W, C, device=DEV, dtype=torch.bfloat16)
    w = (torch.randn(C, C, device=DEV) * C ** -0.5).bfloat16()
    b = torch.randn(C, device=DEV, dtype=torch.bfloat16)
    with torch.no_grad():
        o = linear_residual(t, w, b, res.permute(0, 2, 3, 1)).permute(0, 3, 1, 2)
        ref = _ref(t, w, b, res.permute(0, 2, 3, 1)).permute(0, 3, 1, 2)
        assert (o.float() - ref).abs().max().item() < 0.05 * ref.abs().max().item()
        g = torch.cuda.CUDAGraph()
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            with torch.cuda.graph(g):
                og = linear_residual(t, w, b, res.permute(0, 2, 3, 1))
        torch.cuda.current_stream().wait_stream(s)
        res.mul_(2)  # replay reads the live residual
        g.replay()
        torch.cuda.synchronize()
        ref2 = _ref(t, w, b, res.permute(0, 2, 3, 1))
        assert (og.float() - ref2).abs().max().item() < 0.05 * ref2.abs().max().item()


def test_unet_transformer_fused_residuals_match_unfused(monkeypatch):
    from kubernetes_cloud_amd.models import unet
    torch.manual_seed(1)
    m = unet.Transformer2DModel(320, 8, 768).to(DEV).bfloat16().eval()
    for p_ in m.parameters():
        torch.nn.init.normal_(p_, std=0.05)
    x = torch.randn(2, 320, 32, 32, device=DEV, dtype=torch.bfloat16).contiguous(memory_format=torch.channels_last)
    ctx = torch.randn(2, 77, 768, device=DEV, dtype=torch.bfloat16)
    with torch.no_grad():
        fused = m(x, ctx)
        monkeypatch.setattr(unet, "_FUSE_RES", False)
        plain = m(x, ctx)
    assert _lib.has("kca_gemm_lt")
    err = (fused.float() - plain.float()).abs().max().item()
    assert err < 0.03 * plain.float().abs().max().item(), err
