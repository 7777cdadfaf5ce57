"""Horovod Adasum (resnet50_horovod.py:115-139, op=hvd.Adasum) as a DDP comm
hook over gloo: the recursive-doubling result equals the pairwise Adasum tree
computed directly from every rank's gradient, is bitwise identical on all
ranks, reduces to the mean-free sum for orthogonal gradients and to the
gradient itself for identical ones, and the ResNet trainer runs with it."""
import os
import tempfile

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from kubernetes_cloud_amd.train.resnet import adasum_pair


def _port():
    # a file store: no TCP port to race for when the suite runs under pytest-xdist
    fd, path = tempfile.mkstemp(prefix="kca_adasum_")
    os.close(fd)
    os.unlink(path)
    return path


def _grads(world, n=300, seed=0):
    g = torch.Generator().manual_seed(seed)
    return [torch.randn(n, generator=g) for _ in range(world)]


def _seg(n=300):
    return torch.cat([torch.full((100,), 0), torch.full((150,), 1), torch.full((50,), 2)]).long(), 3


def _worker(rank, world, port, q):
    dist.init_process_group("gloo", init_method=f"file://{port}", rank=rank, world_size=world)
    from kubernetes_cloud_amd.train.resnet import adasum_allreduce
    buf = _grads(world)[rank].clone()
    seg, n = _seg()
    adasum_allreduce(buf, seg, n)
    q.put((rank, buf))
    dist.barrier()
    dist.destroy_process_group()


def _hier_worker(rank, world, port, q):
    dist.init_process_group("gloo", init_method=f"file://{port}", rank=rank, world_size=world)
    from kubernetes_cloud_amd.train.resnet import adasum_groups, hierarchical_adasum
    lg, cg = adasum_groups(world, rank, 2)
    buf = _grads(world)[rank].clone()
    seg, n = _seg()
    hierarchical_adasum(buf, seg, n, lg, cg)
    q.put((rank, buf))
    dist.barrier()
    dist.destroy_process_group()


def test_hierarchical_adasum_averages_in_node_then_adasum_across():
    """Horovod's GPU Adasum (resnet50_horovod.py:121-123): 2 nodes x 2 local ranks ->
    Adasum(mean(g0, g1), mean(g2, g3)) on every rank (the LR is scaled by the local size)."""
    world = 4
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    ps = [ctx.Process(target=_hier_worker, args=(r, world, port, q)) for r in range(world)]
    for p in ps:
        p.start()
    res = dict(q.get(timeout=400) for _ in ps)
    for p in ps:
        p.join(timeout=300)
        assert p.exitcode == 0
    seg, n = _seg()
    g = _grads(world)
    ref = adasum_pair((g[0] + g[1]) / 2, (g[2] + g[3]) / 2, seg, n)
    for r in range(world):
        assert torch.equal(res[r], res[0])
    assert torch.allclose(res[0], ref, atol=1e-5)


def _tree(gs, seg, n):
    while len(gs) > 1:
        gs = [adasum_pair(gs[i], gs[i + 1], seg, n) for i in range(0, len(gs), 2)]
    return gs[0]


@pytest.mark.parametrize("world", [2, 4])
def test_adasum_recursive_doubling_matches_tree(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    ps = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in ps:
        p.start()
    res = dict(q.get(timeout=400) for _ in ps)
    for p in ps:
        p.join(timeout=300)
        assert p.exitcode == 0
    seg, n = _seg()
    ref = _tree(_grads(world), seg, n)
    for r in range(world):
        assert torch.equal(res[r], res[0])
    assert torch.allclose(res[0], ref, atol=1e-5)


def test_adasum_pair_limits():
    seg, n = _seg()
    a = torch.randn(300)
    assert torch.allclose(adasum_pair(a, a.clone(), seg, n), a, atol=1e-6)  # identical -> the gradient
    b = torch.zeros(300)
    b[:100] = torch.randn(100)
    a2 = a.clone()
    a2[:100] = 0  # orthogonal per segment -> plain sum
    assert torch.allclose(adasum_pair(a2, b, seg, n), a2 + b, atol=1e-6)


def test_resnet_trainer_with_adasum(tmp_path):
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    cmd = [sys.executable, "-m", "kubernetes_cloud_amd.launch", "--num_gpus", "2", "-m",
           "kubernetes_cloud_amd.train.resnet", "--synthetic", "8", "--batch-size", "2", "--epochs", "1",
           "--max-steps", "2", "--use-adasum", "--no-cuda", "--log-dir", str(tmp_path / "logs"),
           "--train-crop-size", "64", "--val-crop-size", "64", "--workers", "0", "--num-classes", "10"]
    env = dict(os.environ, PYTHONPATH=root, CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="")
    r = subprocess.run(cmd, cwd=root, env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    assert "Test Epoch: 1" in r.stdout
