"""Process-group bootstrap: one process per GPU, ``torch.distributed`` over RCCL.

Replaces the reference's launch runtimes (deepspeed.launcher.runner,
accelerate launch, torchrun, mpirun/Horovod -- SURVEY §1 L3) with the
torchrun env:// contract (RANK, LOCAL_RANK, WORLD_SIZE, MASTER_ADDR/PORT).
Backend "nccl" is RCCL on ROCm (xGMI inside a node); "gloo" is used for the
CPU test-suite. ``HSA_ENABLE_IPC_MODE_LEGACY=0`` is required on this pool for
RCCL peer mappings (dmabuf IPC) and is set if absent.

The reference's world-size fallback overwrote a valid distributed world size
with 1 (finetuner-workflow/finetuner/finetuner.py:336-341); here the env is the
single source of truth.
"""
from __future__ import annotations

import datetime
import os
from dataclasses import dataclass

import torch
import torch.distributed as dist


@dataclass
class DistInfo:
    rank: int = 0
    local_rank: int = 0
    world_size: int = 1
    backend: str = "none"

    @property
    def is_main(self) -> bool:
        return self.rank == 0

    @property
    def distributed(self) -> bool:
        return self.world_size > 1


_INFO = DistInfo()


def env_world() -> tuple[int, int, int]:
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", os.environ.get("LOCAL_PROCESS_RANK", "0")))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    return rank, local, world


def init_distributed(backend: str | None = None, timeout_s: int = 1800) -> DistInfo:
    """Initialise the default process group from the env (idempotent)."""
    global _INFO
    rank, local, world = env_world()
    os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    from . import shared_gpu
    shared = shared_gpu.enabled() and torch.cuda.is_available()
    if shared:  # rehearsal: every rank on cuda:0, gloo, device collectives staged through the host
        torch.cuda.set_device(0)
        backend = "gloo"
    if backend is None:
        backend = "nccl" if torch.cuda.is_available() else "gloo"
    if torch.cuda.is_available() and backend == "nccl":
        torch.cuda.set_device(local % max(1, torch.cuda.device_count()))
    if world > 1 and not dist.is_initialized():
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29500")
        kw = {}
        if backend == "nccl":
            kw["device_id"] = torch.device("cuda", torch.cuda.current_device())
        dist.init_process_group(backend=backend, timeout=datetime.timedelta(seconds=timeout_s), **kw)
    if shared and world > 1:
        shared_gpu.install()
    _INFO = DistInfo(rank=rank, local_rank=local, world_size=world,
                     backend=backend if world > 1 else "none")
    return _INFO


def info() -> DistInfo:
    return _INFO


def barrier():
    if dist.is_initialized():
        dist.barrier()


def all_reduce_max(x: float, device=None) -> float:
    if not dist.is_initialized():
        return x
    t = torch.tensor([x], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def all_reduce_sum(x: float, device=None) -> float:
    if not dist.is_initialized():
        return x
    t = torch.tensor([x], dtype=torch.float64, device=device)
    dist.all_reduce(t)
    return float(t.item())


def destroy():
    if dist.is_initialized():
        dist.destroy_process_group()
