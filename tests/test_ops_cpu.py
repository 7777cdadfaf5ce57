"""CPU paths of the round-2 helper ops (their GPU kernels are covered in tests/test_kernels_gpu.py):
split-K weight-gradient policy and math, column sums, fused residual + bias add, and the decode
workspace layout (fan-in counters at its head)."""
import torch

from kubernetes_cloud_amd import ops
from kubernetes_cloud_amd.ops import decode as dops
from kubernetes_cloud_amd.ops.linear import _LinearSplitKW, _wgrad_splits, column_sum, linear_splitk_wgrad


def test_wgrad_split_policy():
    assert _wgrad_splits(65536, 320, 320) == 16
    assert _wgrad_splits(16384, 640, 640) == 8
    assert _wgrad_splits(16384, 5120, 640) == 1   # big outputs fill the chip unsplit
    assert _wgrad_splits(4096, 1280, 1280) == 1   # short reductions stay one GEMM
    assert _wgrad_splits(65536 + 2048 * 3, 320, 320) in (1, 2, 4, 8, 16)
    t = 3 * 8192
    s = _wgrad_splits(t, 320, 320)
    assert s > 1 and t % s == 0


def test_splitk_linear_backward_matches_linear():
    torch.manual_seed(0)
    x = torch.randn(8, 4096, 32, dtype=torch.float64, requires_grad=True)
    w = torch.randn(16, 32, dtype=torch.float64, requires_grad=True)
    b = torch.randn(16, dtype=torch.float64, requires_grad=True)
    y = _LinearSplitKW.apply(x, w, b)  # 32768 tokens: split path
    g = torch.randn_like(y)
    y.backward(g)
    x2, w2, b2 = (t.detach().clone().requires_grad_() for t in (x, w, b))
    torch.nn.functional.linear(x2, w2, b2).backward(g)
    torch.testing.assert_close(x.grad, x2.grad)
    torch.testing.assert_close(w.grad, w2.grad, rtol=1e-6, atol=1e-4)  # fp32 partial sums
    torch.testing.assert_close(b.grad, b2.grad)
    # off the GPU the public entry point is plain F.linear
    assert linear_splitk_wgrad(x.detach(), w.detach()).shape == (8, 4096, 16)


def test_column_sum_cpu_fallback():
    x = torch.randn(100, 24).to(torch.bfloat16)
    torch.testing.assert_close(column_sum(x).float(), x.sum(0).float())


def test_add_bias_nhwc_cpu_fallback():
    a = torch.randn(2, 16, 3, 3).to(torch.bfloat16).to(memory_format=torch.channels_last)
    b = torch.randn_like(a)
    bias = torch.randn(16)
    ref = a.float() + b.float() + bias[None, :, None, None]
    torch.testing.assert_close(ops.add_bias_nhwc(a, b, bias).float(), ref, rtol=1e-2, atol=2e-2)
    torch.testing.assert_close(ops.add_bias_nhwc(a, None, bias).float(), a.float() + bias[None, :, None, None],
                               rtol=1e-2, atol=2e-2)


def test_decode_workspace_reserves_fanin_counters():
    B, H, Hkv, D, L = 3, 16, 16, 256, 2048
    chunk = 64
    ns = -(-L // chunk)
    n = dops.decode_ws_floats(B, H, Hkv, D, L, chunk)
    cw = -(-(B * H) // 4) * 4
    assert n == cw + B * H * ns * (D + 2)
    assert cw % 4 == 0 and cw >= B * H  # 16-B aligned partials after the counters
    assert dops.decode_ws_floats(B, H, Hkv, D, 64, 64) == 0  # one split: no workspace
