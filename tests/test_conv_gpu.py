"""The matrix-core 3x3 convolution (ops/conv.py, csrc/kernels/conv_igemm.hip) against an fp32 PyTorch
convolution: the SD-1.5 UNet shapes' channel counts (multiples of 64, Cout 320 = 2.5 N tiles), the
padding rows of every tap, bias, a batch whose pixel blocks span images, and the autograd path
(forward native, backward PyTorch's)."""
import pytest
import torch

pytestmark = pytest.mark.gpu

dev = torch.device("cuda", 0)


def _cl(t):
    return t.contiguous(memory_format=torch.channels_last)


@pytest.mark.parametrize("N,H,W,C,Co,bias", [(2, 8, 8, 64, 64, False), (1, 16, 8, 128, 192, True),
                                             (3, 8, 16, 64, 320, True), (2, 32, 32, 320, 320, False),
                                             (1, 16, 16, 640, 1280, True)])
def test_conv3x3_matches_fp32(N, H, W, C, Co, bias):
    from kubernetes_cloud_amd.ops import _lib
    from kubernetes_cloud_amd.ops import conv as kconv
    from kubernetes_cloud_amd.ops.conv import conv3x3, conv3x3_reference, supported
    _lib.require()
    kconv._MODE = "all"
    g = torch.Generator(device=dev).manual_seed(N * 1000 + C + Co)
    x = _cl(torch.randn(N, C, H, W, device=dev, generator=g).bfloat16())
    w = _cl((torch.randn(Co, C, 3, 3, device=dev, generator=g) / (3 * C ** 0.5)).bfloat16())
    b = (0.1 * torch.randn(Co, device=dev, generator=g)).bfloat16() if bias else None
    assert supported(x, w)
    y = conv3x3(x, w, b)
    assert y.is_contiguous(memory_format=torch.channels_last) and y.shape == (N, Co, H, W)
    ref = conv3x3_reference(x, w, b)
    err = (y.float() - ref).abs().max().item()
    assert err <= 2e-2 * ref.abs().max().item() + 1e-3, err


def test_conv3x3_autograd_backward_is_pytorchs():
    from kubernetes_cloud_amd.ops import conv as kconv
    from kubernetes_cloud_amd.ops.conv import conv3x3
    kconv._MODE = "all"
    g = torch.Generator(device=dev).manual_seed(7)
    x = _cl(torch.randn(2, 64, 8, 8, device=dev, generator=g).bfloat16()).requires_grad_()
    w = _cl((torch.randn(128, 64, 3, 3, device=dev, generator=g) / 24).bfloat16()).requires_grad_()
    b = (0.1 * torch.randn(128, device=dev, generator=g)).bfloat16().requires_grad_()
    gy = _cl(torch.randn(2, 128, 8, 8, device=dev, generator=g).bfloat16())
    conv3x3(x, w, b).backward(gy)
    x2, w2, b2 = (t.detach().clone().requires_grad_() for t in (x, w, b))
    torch.nn.functional.conv2d(x2, w2, b2, padding=1).backward(gy)
    for a_, r_ in ((x.grad, x2.grad), (w.grad, w2.grad), (b.grad, b2.grad)):
        assert (a_.float() - r_.float()).abs().max().item() <= 2e-2 * r_.float().abs().max().item() + 1e-2
