"""CPU test of the shared-GPU rehearsal shim (parallel/shared_gpu.py): with
host staging forced onto CPU tensors, the ZeRO engine at world 2 must still
match the one-process run, i.e. every patched collective (reduce-scatter,
all-gather-into-tensor, all-reduce, async work handles) is exact."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from .test_dist_gloo import _batches, _model, _reference


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, stage, out_path):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.set_num_threads(1)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from kubernetes_cloud_amd.parallel import shared_gpu
    shared_gpu.install(force=True)
    assert dist.all_reduce is not shared_gpu._ORIG["all_reduce"]
    from kubernetes_cloud_amd.train.engine import TrainEngine
    m = _model()
    m.train()
    eng = TrainEngine(m, lr=1e-2, weight_decay=0.01, zero_stage=stage, grad_accum=2, bucket_elems=3_000)
    for step in _batches(world, 2):
        mbs = [b[rank * 2:(rank + 1) * 2] for b in step]
        eng.train_batch(mbs, lambda ids: m(ids, labels=ids))
    with eng.gathered():
        sd = {k: v.detach().clone() for k, v in m.state_dict().items()}
    if rank == 0:
        torch.save(sd, out_path)
    dist.barrier()
    shared_gpu.uninstall()
    dist.destroy_process_group()


@pytest.mark.parametrize("stage", [1, 2, 3])
def test_staged_collectives_keep_zero_exact(stage, tmp_path):
    out = str(tmp_path / f"sd{stage}.pt")
    ctx = mp.get_context("spawn")
    port = _port()
    ps = [ctx.Process(target=_worker, args=(r, 2, port, stage, out)) for r in range(2)]
    for p in ps:
        p.start()
    for p in ps:
        p.join(timeout=300)
        assert p.exitcode == 0
    got = torch.load(out, weights_only=True)
    ref = _reference(2)
    for k in ref:
        assert torch.allclose(got[k], ref[k], atol=2e-5, rtol=1e-4), k


def test_shim_disabled_by_default(monkeypatch):
    from kubernetes_cloud_amd.parallel import shared_gpu
    monkeypatch.delenv(shared_gpu.ENV, raising=False)
    assert not shared_gpu.enabled()
    monkeypatch.setenv(shared_gpu.ENV, "1")
    assert shared_gpu.enabled()


def _p2p_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.set_num_threads(1)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from kubernetes_cloud_amd.parallel import shared_gpu
    shared_gpu.install(force=True)
    from kubernetes_cloud_amd.train.resnet import adasum_allreduce
    peer = 1 - rank
    mine = torch.full((5,), float(rank + 1))
    got = torch.zeros(5)
    ops = [dist.P2POp(dist.isend, mine, peer), dist.P2POp(dist.irecv, got, peer)]  # P2POp accepts the originals
    for w in dist.batch_isend_irecv(ops):
        w.wait()
    g = torch.Generator().manual_seed(rank)
    buf = torch.randn(40, generator=g)
    adasum_allreduce(buf, torch.zeros(40, dtype=torch.long), 1)  # Adasum's recursive doubling, staged
    fut = dist.all_reduce(torch.ones(3), async_op=True).get_future()  # DDP comm-hook pattern
    q.put((rank, got.tolist(), buf.tolist(), fut.wait()[0].tolist()))
    dist.barrier()
    shared_gpu.uninstall()
    dist.destroy_process_group()


def test_staged_point_to_point_and_hook_futures():
    """batch_isend_irecv (pipeline stages, Adasum pairs) and async all_reduce futures (DDP comm
    hooks) through the host-staging shim."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    ps = [ctx.Process(target=_p2p_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    res = dict((r[0], r[1:]) for r in (q.get(timeout=120) for _ in ps))
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert res[0][0] == [2.0] * 5 and res[1][0] == [1.0] * 5
    assert res[0][1] == res[1][1]  # Adasum leaves identical bits on both ranks
    assert res[0][2] == [2.0] * 3
