"""Custom xGMI all-reduce (csrc/comm/xgmi_allreduce.hip): two ranks on the
box's single GPU exchange hipIpc handles (gloo bootstrap) and must produce the
exact bf16 sum (and, for the all-gather interleaved into the same call
sequence, the exact concatenation).

The stress case interleaves sizes below and above the one-shot/two-shot switch
and the block-count cap (so the slice->block map changes from call to call),
never synchronises between calls, and makes one rank sleep before its read
phase: with round 1's per-block parity counters a fast rank could overwrite a
staging region the slow rank was still reading; with one
per-rank sequence word every call must stay bit-exact. Sums of small integers
are exact in bf16, so the check is equality."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu

SIZES = (8, 14336, 1 << 20, 8, 14336 * 4, 1 << 21, 65536, 14336, 3 * (1 << 19) + 8, 8, 1 << 18, 14336 * 32)


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _inputs(world, n, it):
    g = torch.Generator().manual_seed(1000 * it + n)
    return [torch.randint(-8, 8, (n,), generator=g).to(torch.bfloat16) for _ in range(world)]


def _tails(rank, world, ar):
    """kca_ar_res_ln (batch 1) and kca_ar_res_stats (M rows) against fp32: the all-reduced partials +
    bias + residual, rounded once (bit-exact: same summation order), then LayerNorm / row statistics
    of the kernel's own rounded stream."""
    import torch.nn.functional as F

    from kubernetes_cloud_amd.ops.skinny_mm import RowStatsBuf, row_stats_reference
    errs = []
    for N in (1024, 14336):
        for two in (False, True):
            g = torch.Generator().manual_seed(N + two)
            ts = [(0.5 * torch.randn(N, generator=g)).bfloat16() for _ in range(world)]
            h = (2 * torch.randn(N, generator=g)).bfloat16()
            bias = (0.1 * torch.randn(N, generator=g)).bfloat16()
            gam = [(1 + 0.1 * torch.randn(N, generator=g)).bfloat16() for _ in range(2)]
            bet = [(0.1 * torch.randn(N, generator=g)).bfloat16() for _ in range(2)]
            d = "cuda"
            h_out, xn, xn2 = (torch.empty(N, device=d, dtype=torch.bfloat16) for _ in range(3))
            ar.res_ln(ts[rank].to(d), bias.to(d), h.to(d), h_out, gam[0].to(d), bet[0].to(d), 1e-5, xn,
                      *((gam[1].to(d), bet[1].to(d), xn2) if two else ()))
            torch.cuda.synchronize()
            ref_h = (h.float() + (sum(t.float() for t in ts) + bias.float())).bfloat16()
            errs.append(float((h_out.cpu().float() - ref_h.float()).abs().max()))
            ho = h_out.cpu().float()
            for gm, bt, out in ((gam[0], bet[0], xn),) + (((gam[1], bet[1], xn2),) if two else ()):
                ref = F.layer_norm(ho, (N,), gm.float(), bt.float(), 1e-5)
                errs.append(max(0.0, float((out.cpu().float() - ref).abs().max()) - 0.05))
        for M in (3, 32):
            g = torch.Generator().manual_seed(7 * M + N)
            ts = [(0.5 * torch.randn(M, N, generator=g)).bfloat16() for _ in range(world)]
            h = (2 * torch.randn(M, N, generator=g) + 1).bfloat16()
            bias = (0.1 * torch.randn(N, generator=g)).bfloat16()
            st = RowStatsBuf(M, N, "cuda")
            hb = h.cuda()
            ar.res_stats(ts[rank].cuda(), bias.cuda(), hb, hb, st, 1e-5)  # in place, as the decode layer runs it
            torch.cuda.synchronize()
            ref_h = (h.float() + (sum(t.float() for t in ts) + bias.float())).bfloat16()
            errs.append(float((hb.cpu().float() - ref_h.float()).abs().max()))
            ref_st = row_stats_reference(hb.cpu(), 1e-5)
            rel = ((st.merged(M).cpu() - ref_st).abs() / (ref_st.abs() + 1e-3)).max()
            errs.append(max(0.0, float(rel) - 1e-4))
    return errs


def _worker(rank, world, port, q, mode):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), HSA_ENABLE_IPC_MODE_LEGACY="0")
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.cuda.set_device(0)
    from kubernetes_cloud_amd.parallel.custom_ar import ONE_SHOT, TWO_SHOT, AllReduceError, XGMIAllReduce
    try:
        if mode == "tails":
            ar = XGMIAllReduce(None, max_bytes=4 << 20, spin_limit=1 << 24)
            errs = _tails(rank, world, ar)
            q.put((rank, ar.error() == 0 and ar.res_ln_calls == 4 and ar.res_stats_calls == 4, errs))
            dist.barrier()
            ar.close()
            return
        if mode == "timeout":
            ar = XGMIAllReduce(None, max_bytes=1 << 20, spin_limit=4000)
            ok = True
            if rank == 0:  # rank 1 never joins: the kernel must time out, poison and flag
                t = torch.ones(4096, device="cuda", dtype=torch.bfloat16)
                ar.all_reduce_(t)
                torch.cuda.synchronize()
                ok = bool(torch.isnan(t.float()).all())
                try:
                    ar.check()
                    ok = False
                except AllReduceError:
                    pass
            q.put((rank, ok, []))
            dist.barrier()
            ar.close()
            return
        ar = XGMIAllReduce(None, max_bytes=8 << 20, one_shot_max=64 << 10, spin_limit=1 << 24)
        outs, refs = [], []
        for rep in range(3):
            for it, n in enumerate(SIZES):
                xs = _inputs(world, n, it)
                t = xs[rank].cuda()
                # rank 1 lags before its read phase on every other call
                ar.debug_delay = 300 if (rank == 1 and (it + rep) % 2 == 0) else 0
                algo = None if rep == 0 else (ONE_SHOT if rep == 1 and n * 2 <= (8 << 20) else TWO_SHOT)
                ar.all_reduce_(t, algo=algo)
                outs.append(t)
                refs.append(sum(x.float() for x in xs))
                if n * 2 <= (8 << 20) and it % 3 == 0:  # all-gathers share the call sequence
                    g = xs[rank].cuda() + 1
                    outs.append(ar.all_gather(g))
                    refs.append(torch.cat([x.float() + 1 for x in xs]))
        torch.cuda.synchronize()
        errs = [float((o.float().cpu() - r).abs().max()) for o, r in zip(outs, refs)]
        q.put((rank, ar.error() == 0, errs))
        dist.barrier()
        ar.close()
    finally:
        dist.destroy_process_group()


def _run(mode):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    ps = [ctx.Process(target=_worker, args=(r, 2, port, q, mode)) for r in range(2)]
    for p in ps:
        p.start()
    res = [q.get(timeout=240) for _ in range(2)]
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    return res


def test_xgmi_allreduce_interleaved_sizes_with_rank_skew_is_exact():
    for rank, no_err, errs in _run("stress"):
        assert no_err, rank
        assert errs and max(errs) == 0.0, (rank, errs)


def test_xgmi_allreduce_timeout_poisons_and_raises():
    for rank, ok, _ in _run("timeout"):
        assert ok, rank


def test_xgmi_fused_tails_match_fp32():
    """The TP decode layer's all-reduce tails: residual + bias + LayerNorm (batch 1, with and without the
    second LayerNorm) and residual + bias + row statistics (M rows), N = 1024 and BLOOM's 14336."""
    for rank, ok, errs in _run("tails"):
        assert ok, rank
        assert max(errs) == 0.0, (rank, errs)
