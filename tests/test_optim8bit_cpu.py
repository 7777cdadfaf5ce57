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
