"""Custom one-shot all-reduce (csrc/comm/xgmi_allreduce.hip): two ranks on the
box's single GPU exchange hipIpc handles (gloo bootstrap) and must produce the
exact bf16 sum, repeatedly (double-buffer parity, device-side call counters)."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), HSA_ENABLE_IPC_MODE_LEGACY="0")
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.cuda.set_device(0)
    from kubernetes_cloud_amd.parallel.custom_ar import XGMIAllReduce
    ar = XGMIAllReduce(None, max_bytes=1 << 20, spin_limit=1 << 22)
    errs = []
    for it, n in enumerate((8, 14336, 4 * 14336, 65536, 14336)):
        g = torch.Generator().manual_seed(1000 * it)
        xs = [torch.randint(-8, 8, (n,), generator=g).to(torch.bfloat16) for _ in range(world)]
        t = xs[rank].cuda()
        ar.all_reduce_(t)
        torch.cuda.synchronize()
        ref = sum(x.float() for x in xs)
        errs.append(float((t.float().cpu() - ref).abs().max()))
    q.put((rank, errs, ar.error()))
    dist.barrier()
    ar.close()
    dist.destroy_process_group()


def test_one_shot_allreduce_two_ranks_one_gpu():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    ps = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    res = [q.get(timeout=240) for _ in range(2)]
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, errs, err_flag in res:
        assert err_flag == 0, (rank, err_flag)
        assert max(errs) == 0.0, (rank, errs)
