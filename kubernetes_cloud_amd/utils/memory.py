"""Memory telemetry (what finetuner-workflow/finetuner/utils.py:28-108 reports):
GPU free/used from the HIP runtime (``hipMemGetInfo`` via torch), torch's
allocator view (allocated / reserved / peak) and host RSS / free RAM."""
from __future__ import annotations

import dataclasses
import os
import resource

import torch


def _gib(x: float) -> str:
    return f"{x / 2**30:.2f}GiB"


@dataclasses.dataclass
class GPUMem:
    free: int
    total: int

    @property
    def used(self) -> int:
        return self.total - self.free

    def __str__(self):
        return f"gpu used={_gib(self.used)} free={_gib(self.free)} total={_gib(self.total)}"


@dataclasses.dataclass
class TorchMem:
    allocated: int
    reserved: int
    peak: int

    @property
    def used(self) -> int:
        return self.allocated

    def __str__(self):
        return f"torch alloc={_gib(self.allocated)} reserved={_gib(self.reserved)} peak={_gib(self.peak)}"


@dataclasses.dataclass
class CPUMem:
    maxrss: int
    free: int | None

    def __str__(self):
        f = _gib(self.free) if self.free is not None else "?"
        return f"cpu maxrss={_gib(self.maxrss)} free={f}"


@dataclasses.dataclass
class MemoryUsage:
    gpu: GPUMem | None
    torch: TorchMem | None
    cpu: CPUMem

    @classmethod
    def now(cls, device=None) -> "MemoryUsage":
        gpu = tm = None
        if torch.cuda.is_available():
            dev = device if device is not None else torch.cuda.current_device()
            free, total = torch.cuda.mem_get_info(dev)
            gpu = GPUMem(free, total)
            tm = TorchMem(torch.cuda.memory_allocated(dev), torch.cuda.memory_reserved(dev),
                          torch.cuda.max_memory_allocated(dev))
        rss = resource.getrusage(resource.RUSAGE_SELF).ru_maxrss * 1024
        try:
            import psutil
            free = psutil.virtual_memory().available
        except Exception:  # pragma: no cover
            free = None
        return cls(gpu, tm, CPUMem(rss, free))

    def __str__(self):
        parts = [str(p) for p in (self.gpu, self.torch, self.cpu) if p is not None]
        return " | ".join(parts)


def host_info() -> dict:
    info = {"pid": os.getpid(), "torch": torch.__version__, "hip": getattr(torch.version, "hip", None)}
    if torch.cuda.is_available():
        p = torch.cuda.get_device_properties(0)
        info.update(gpu=p.name, arch=getattr(p, "gcnArchName", ""), cus=p.multi_processor_count,
                    hbm_gib=round(p.total_memory / 2**30, 1), n_gpus=torch.cuda.device_count())
    return info
