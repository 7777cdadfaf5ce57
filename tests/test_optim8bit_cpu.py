"""Block-wise 8-bit AdamW (N10): CPU math, quantisation error bounds and
convergence against fp32 AdamW on a least-squares problem."""
import torch

from kubernetes_cloud_amd.train.optim import FlatAdamW, FlatAdamW8bit


def test_quant_roundtrip_error_bounds():
    torch.manual_seed(0)
    n = 2048 * 3
    o = FlatAdamW8bit(torch.zeros(n))
    m = torch.randn(n) * torch.logspace(-4, 0, n)
    v = torch.rand(n) * torch.logspace(-8, 0, n)
    o._quant(m, v)
    mq, vq = o.dequant()
    # companded codes: relative error of the block max <= 1/127 scale steps
    for blk in range(3):
        sl = slice(blk * 2048, (blk + 1) * 2048)
        am = m[sl].abs().max()
        assert (mq[sl] - m[sl]).abs().max() <= 2 * am / 127 + 1e-12
        av = v[sl].max()
        assert (vq[sl] - v[sl]).abs().max() <= 4 * av / 255 + 1e-12
    assert o.m_codes.dtype == torch.int8 and o.v_codes.dtype == torch.uint8


def test_8bit_adamw_converges_like_fp32():
    torch.manual_seed(1)
    A = torch.randn(256, 64)
    x_true = torch.randn(64)
    y = A @ x_true
    res = {}
    for name, cls in (("fp32", FlatAdamW), ("int8", FlatAdamW8bit)):
        x = torch.zeros(64)
        opt = cls(x, lr=5e-2)
        for _ in range(300):
            r = A @ opt.master - y
            opt.grad.copy_(A.t() @ r / 256)
            opt.step()
        res[name] = float((A @ opt.master - y).pow(2).mean())
    assert res["fp32"] < 1e-3
    assert res["int8"] < 1e-2, res


def test_state_dict_roundtrip():
    o = FlatAdamW8bit(torch.randn(4096), lr=1e-3)
    o.grad.normal_()
    o.step()
    sd = {k: (v.clone() if torch.is_tensor(v) else v) for k, v in o.state_dict().items()}
    o2 = FlatAdamW8bit(o.master.clone(), lr=1e-3)
    o2.load_state_dict(sd)
    assert torch.equal(o2.m_codes, o.m_codes) and o2.step_count == 1


def test_host_offload_adamw_matches_device_math():
    """HostOffloadAdamW (pinned host state + AVX host AdamW, N2) == FlatAdamW."""
    from kubernetes_cloud_amd.io import native
    from kubernetes_cloud_amd.train.optim import HostOffloadAdamW
    if not native.available():
        import pytest
        pytest.skip("libkca_host.so not built")
    torch.manual_seed(2)
    n = 64 * 300
    p0 = torch.randn(n)
    mask = (torch.arange(n // 64) % 2).to(torch.uint8)
    bf = [torch.empty(n, dtype=torch.bfloat16) for _ in range(2)]
    a = FlatAdamW(p0.clone(), lr=1e-2, weight_decay=0.1, wd_mask=mask, model_bf16=bf[0])
    HostOffloadAdamW.CHUNK = 64 * 70  # several pipeline chunks, ragged tail
    b = HostOffloadAdamW(p0.clone(), lr=1e-2, weight_decay=0.1, wd_mask=mask, model_bf16=bf[1])
    for it in range(4):
        g = torch.randn(n)
        a.grad.copy_(g)
        b.grad.copy_(g)
        for o in (a, b):
            o.set_clip(o.local_sumsq(), 1.0)
            o.step(use_clip=True)
    assert torch.allclose(a.master, b.master, atol=1e-6, rtol=1e-5)
    assert torch.allclose(a.exp_avg_sq, b.exp_avg_sq, atol=1e-7, rtol=1e-5)
    assert torch.equal(bf[1], b.master.bfloat16())
