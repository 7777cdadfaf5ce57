"""Batched-decode MFMA GEMM (csrc/kernels/skinny_mfma.hip) against fp32 PyTorch references:
plain / bias+GELU / residual + row-stats tail / LN-on-load / two jobs / two K-parts, bf16 and fp16,
M = 2..64, every launch-shape variant (one or two weight tiles per wave, K split over 1..16 workgroups)."""
import pytest
import torch

from kubernetes_cloud_amd.ops import skinny_mm as sm

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.fixture(autouse=True)
def _producer_merged_stats(monkeypatch):
    """These tests read RowStatsBuf.stats: the producer-merged (last-arriver) tails. The consumer-merged
    default is covered by test_consumer_merged_row_stats and the engine tests."""
    monkeypatch.setattr(sm, "STATS_CONSUMER", False)


def _close(a, b, tol):
    a, b = a.float(), b.float()
    err = (a - b).abs().max().item()
    scale = b.abs().max().item() + 1e-6
    assert err <= tol * scale, (err, scale)


def _w(N, K, dt, g):
    return (torch.randn(N, K, generator=g, device=DEV) / K ** 0.5).to(dt)


@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("M", [2, 3, 4, 8, 16, 17, 32, 33, 64])
@pytest.mark.parametrize("NK", [(1024, 4096), (4096, 1792), (1360, 1000), (640, 6208)])
def test_mm_plain_bias_gelu(dt, M, NK):
    """(K >= 6144 at M >= 17: the 8-wave, 128-wide-chunk workgroups of the long-K plan)"""
    N, K = NK
    g = torch.Generator(device=DEV).manual_seed(M * 7 + N)
    x = torch.randn(M, K, generator=g, device=DEV).to(dt)
    w = _w(N, K, dt, g)
    b = (0.1 * torch.randn(N, generator=g, device=DEV)).to(dt)
    for act in (0, 1, 2):
        y = sm.mm(x, w, b, act)
        _close(y, sm.mm_reference([(x, w, None)], b, act, dtype=dt), 1.5e-2)


@pytest.mark.parametrize("M", [2, 8, 24, 64])
@pytest.mark.parametrize("ks,nr", [(1, 1), (3, 1), (16, 1), (1, 2), (8, 2), (0, 2), (0, 1)])
def test_mm_launch_shapes(M, ks, nr):
    g = torch.Generator(device=DEV).manual_seed(3)
    N, K = 2048, 4096
    x = torch.randn(M, K, generator=g, device=DEV).bfloat16()
    w = _w(N, K, torch.bfloat16, g)
    y = torch.empty(M, N, device=DEV, dtype=torch.bfloat16)
    sm.launch([sm.job([sm.part(x, w)], N, y)], M, torch.bfloat16, ks=ks, nr=nr)
    _close(y, sm.mm_reference([(x, w, None)]), 1.5e-2)


@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("M", [2, 5, 16, 32, 64])
@pytest.mark.parametrize("N", [1024, 14336])
def test_residual_tail_then_ln_on_load(dt, M, N):
    """out-projection + bias + residual -> h' with its row stats, then the next projection normalises
    h' on load: against fp32 LayerNorm(h') of the kernel's own rounded h'."""
    g = torch.Generator(device=DEV).manual_seed(M + N)
    K = 1792
    o = torch.randn(M, K, generator=g, device=DEV).to(dt)
    wo = _w(N, K, dt, g)
    bo = (0.1 * torch.randn(N, generator=g, device=DEV)).to(dt)
    h = (3 * torch.randn(M, N, generator=g, device=DEV) + 0.5).to(dt)
    h0 = h.clone()
    st = sm.RowStatsBuf(M, N, DEV)
    for rep in range(2):  # the counters re-arm: a second launch is as good as the first
        h.copy_(h0)
        sm.mm(o, wo, bo, out=h, res=h, stats=st, eps=1e-5)
        ref_h = sm.mm_reference([(o, wo, None)], bo, res=h0, dtype=dt)
        _close(h, ref_h, 1e-2)
        ref_st = sm.row_stats_reference(h, 1e-5)
        torch.testing.assert_close(st.stats[:, 0], ref_st[:, 0], atol=1e-4 * ref_st[:, 0].abs().max().item() + 1e-5,
                                   rtol=1e-4)
        torch.testing.assert_close(st.stats[:, 1], ref_st[:, 1], rtol=1e-4, atol=1e-6)
    gamma = (1 + 0.1 * torch.randn(N, generator=g, device=DEV)).to(dt)
    beta = (0.1 * torch.randn(N, generator=g, device=DEV)).to(dt)
    w2 = _w(3072, N, dt, g)
    b2 = (0.1 * torch.randn(3072, generator=g, device=DEV)).to(dt)
    y = sm.mm(h, w2, b2, act=1, ln=(st.stats, gamma, beta))
    xn = torch.nn.functional.layer_norm(h.float(), (N,), gamma.float(), beta.float(), 1e-5).to(dt)
    _close(y, sm.mm_reference([(xn, w2, None)], b2, 1, dtype=dt), 2e-2)


@pytest.mark.parametrize("M", [3, 16, 40])
def test_two_jobs_and_two_parts(M):
    """GPT-J's layer: [QKV | fc_in+GELU] of LN(h) in one launch, then o.Wo^T + g.Wf^T + b + h (one
    residual job with two K-parts) with the stats tail."""
    dt = torch.bfloat16
    g = torch.Generator(device=DEV).manual_seed(M)
    d, f = 1024, 4096
    h = torch.randn(M, d, generator=g, device=DEV).to(dt)
    st = sm.RowStatsBuf(M, d, DEV)
    st.stats.copy_(sm.row_stats_reference(h, 1e-5))
    gamma = (1 + 0.1 * torch.randn(d, generator=g, device=DEV)).to(dt)
    beta = (0.1 * torch.randn(d, generator=g, device=DEV)).to(dt)
    wq, wi = _w(3 * d, d, dt, g), _w(f, d, dt, g)
    bi = (0.1 * torch.randn(f, generator=g, device=DEV)).to(dt)
    qkv = torch.empty(M, 3 * d, device=DEV, dtype=dt)
    gg = torch.empty(M, f, device=DEV, dtype=dt)
    ln = (st.stats, gamma, beta)
    sm.launch([sm.job([sm.part(h, wq, ln)], 3 * d, qkv), sm.job([sm.part(h, wi, ln)], f, gg, bi, act=1)], M, dt)
    _close(qkv, sm.mm_reference([(h, wq, ln)], dtype=dt), 1.5e-2)
    _close(gg, sm.mm_reference([(h, wi, ln)], bi, 1, dtype=dt), 1.5e-2)
    o = torch.randn(M, d, generator=g, device=DEV).to(dt)
    wo, wf = _w(d, d, dt, g), _w(d, f, dt, g)
    bsum = (0.1 * torch.randn(d, generator=g, device=DEV)).to(dt)
    h0 = h.clone()
    st2 = sm.RowStatsBuf(M, d, DEV)
    sm.launch([sm.job([sm.part(o, wo), sm.part(gg, wf)], d, h, bsum, res=h, stats=st2, eps=1e-5)], M, dt)
    _close(h, sm.mm_reference([(o, wo, None), (gg, wf, None)], bsum, res=h0, dtype=dt), 1e-2)
    torch.testing.assert_close(st2.stats[:, 1], sm.row_stats_reference(h, 1e-5)[:, 1], rtol=1e-4, atol=1e-6)


def test_rejects_bad_shapes():
    x = torch.randn(4, 100, device=DEV).bfloat16()  # K % 8 != 0
    w = torch.randn(64, 100, device=DEV).bfloat16()
    with pytest.raises(RuntimeError):
        sm.mm(x, w)
    x = torch.randn(65, 128, device=DEV).bfloat16()  # M > 64
    w = torch.randn(64, 128, device=DEV).bfloat16()
    with pytest.raises(RuntimeError):
        sm.mm(x, w)


@pytest.mark.parametrize("M", [4, 32])
def test_split_k_is_deterministic(M):
    """The last arriving K slice sums every slice in slice order: repeated launches are bit-identical
    whatever the arrival order (seeded sampling must reproduce under graph replay)."""
    g = torch.Generator(device=DEV).manual_seed(1)
    x = torch.randn(M, 16384, generator=g, device=DEV).bfloat16()
    w = _w(1024, 16384, torch.bfloat16, g)
    outs = []
    for _ in range(20):
        y = torch.empty(M, 1024, device=DEV, dtype=torch.bfloat16)
        sm.launch([sm.job([sm.part(x, w)], 1024, y)], M, torch.bfloat16, ks=16)
        outs.append(y)
    torch.cuda.synchronize()
    assert all(torch.equal(outs[0], o) for o in outs[1:])


@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("M", [2, 8, 16, 32, 64])
@pytest.mark.parametrize("NK", [(1024, 4096), (1360, 1000), (640, 6208), (2052, 1800)])
def test_packed_weight_stream_is_bit_identical(dt, M, NK):
    """The packed stream layout (pack_weight: 16 x 128 sub-tiles, zero-padded rows / columns) feeds the
    same fragments as the row-major weight, so every variant's output is bit-identical -- two K parts,
    the residual + row-stats tail and LN-on-load included -- and matches the fp32 reference."""
    N, K = NK
    g = torch.Generator(device=DEV).manual_seed(M * 13 + N)
    x = torch.randn(M, K, generator=g, device=DEV).to(dt)
    w = _w(N, K, dt, g)
    wp = sm.pack_weight(w)
    assert wp.shape == (-(-N // 16), -(-K // 128), 16, 128)
    b = (0.1 * torch.randn(N, generator=g, device=DEV)).to(dt)
    for act in (0, 1):
        y0 = sm.mm(x, w, b, act)
        y1 = sm.mm(x, w, b, act, packed=wp)
        assert torch.equal(y0, y1)
        _close(y1, sm.mm_reference([(x, w, None)], b, act, dtype=dt), 1.5e-2)
    for kc in (128, 256):  # both chunk widths read the 128-wide sub-tiles
        old = sm._KC
        sm._KC = kc
        try:
            assert torch.equal(sm.mm(x, w, b), sm.mm(x, w, b, packed=wp))
        finally:
            sm._KC = old
    # two K parts into one residual with the row-stats tail, then LN-on-load from those statistics
    if N % 64 == 0:
        K2 = 512
        x2 = torch.randn(M, K2, generator=g, device=DEV).to(dt)
        w2 = _w(N, K2, dt, g)
        h = torch.randn(M, N, generator=g, device=DEV).to(dt)
        outs = []
        for pk in (False, True):
            hb = h.clone()
            st = sm.RowStatsBuf(M, N, DEV)
            parts = [sm.part(x, w, packed=wp if pk else None),
                     sm.part(x2, w2, packed=sm.pack_weight(w2) if pk else None)]
            sm.launch([sm.job(parts, N, hb, b, res=hb, stats=st)], M, dt)
            wn = _w(256, N, dt, g) if not outs else outs[0][2]
            gam = torch.ones(N, device=DEV, dtype=dt)
            y = sm.mm(hb, wn, ln=(st.stats, gam, None), packed=sm.pack_weight(wn) if pk else None)
            outs.append((hb, y, wn))
        assert torch.equal(outs[0][0], outs[1][0]) and torch.equal(outs[0][1], outs[1][1])


@pytest.mark.parametrize("M", [2, 8, 32])
@pytest.mark.parametrize("N", [1024, 14336])
def test_consumer_merged_row_stats(M, N, monkeypatch):
    """Publish-only residual tails (STATS_CONSUMER): the producer writes per-16-column (mean, M2)
    partials and no merged stats; the next projection merges them in its prologue (MmPart.st_nt).
    Its LN-on-load output matches the merged-stats path and the fp32 reference, and the host-side
    merge of the partials matches the rows' statistics."""
    dt = torch.bfloat16
    g = torch.Generator(device=DEV).manual_seed(M + N)
    K = 2048
    x = torch.randn(M, K, generator=g, device=DEV).to(dt)
    w = _w(N, K, dt, g)
    b = (0.1 * torch.randn(N, generator=g, device=DEV)).to(dt)
    h0 = torch.randn(M, N, generator=g, device=DEV).to(dt)
    wn = _w(512, N, dt, g)
    gam = (1 + 0.1 * torch.randn(N, generator=g, device=DEV)).to(dt)
    bet = (0.1 * torch.randn(N, generator=g, device=DEV)).to(dt)
    outs = {}
    for cons in (False, True):
        monkeypatch.setattr(sm, "STATS_CONSUMER", cons)
        hb = h0.clone()
        st = sm.RowStatsBuf(M, N, DEV)
        sm.launch([sm.job([sm.part(x, w)], N, hb, b, res=hb, stats=st, eps=1e-5)], M, dt)
        assert st.nt == (N // 16 if cons else 0)
        y = sm.mm(hb, wn, ln=(st, gam, bet))
        outs[cons] = (hb, y, st.merged(M).clone())
    assert torch.equal(outs[False][0], outs[True][0])
    _close(outs[True][2], sm.row_stats_reference(outs[True][0], 1e-5), 1e-4)
    _close(outs[True][1], outs[False][1], 1e-2)
    ref = sm.mm_reference([(sm.ln_on_load_reference(outs[True][0], sm.row_stats_reference(outs[True][0], 1e-5),
                                                     gam, bet), wn, None)])
    _close(outs[True][1], ref, 1.5e-2)
