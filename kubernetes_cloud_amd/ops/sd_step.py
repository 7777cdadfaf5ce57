"""Fused Stable Diffusion sampler step (``csrc/kernels/sd_step.hip``).

``lms_step`` = classifier-free guidance combine + k-diffusion LMS (Euler: order
1) update + the next step's scaled bf16 UNet input, one pass over the latents.
The CPU / fp32 reference below is the same math as ``models.schedulers``'
``LMSDiscreteScheduler.step`` preceded by the pipeline's CFG combine, and pins
the kernel in ``tests/test_kernels_gpu.py``.

Layout contract: ``eps`` ([2B or B, C, H, W] bf16), ``x`` ([B, C, H, W] fp32) and
``xin`` ([2B or B, ...] bf16) share one memory format (the channels-last UNet
output decides it), so flat memory offsets line up element for element.
"""
from __future__ import annotations

import ctypes

import torch

from . import _lib

PRED = {"epsilon": 0, "v_prediction": 1, "sample": 2}


def lms_step(eps: torch.Tensor, x: torch.Tensor, ring: torch.Tensor, coefs: list[float], newest: int,
             sigma: float, guidance: float | None, prediction_type: str = "epsilon",
             in_scale: float | None = None, xin: torch.Tensor | None = None) -> None:
    """In place: ``ring[newest] = d``; ``x += sum_j coefs[j] * d_{newest-j}``;
    ``xin = bf16(x * in_scale)`` (duplicated for CFG) when given."""
    cfg = guidance is not None
    n = x.numel()
    order = ring.shape[0]
    o = len(coefs)
    if eps.is_cuda and eps.dtype == torch.bfloat16 and _lib.has("kca_sd_lms_step"):
        half = eps[: eps.shape[0] // 2] if cfg else eps
        assert x.dtype == torch.float32 and ring.dtype == torch.float32 and ring.is_contiguous()
        assert half.stride() == x.stride() and (xin is None or xin[: x.shape[0]].stride() == x.stride())
        assert (not cfg or eps.shape[0] == 2 * x.shape[0]) and ring[0].numel() == n
        c = (ctypes.c_float * 4)(*([float(v) for v in coefs] + [0.0] * (4 - o)))
        _lib.call("kca_sd_lms_step", eps.data_ptr(), x.data_ptr(), ring.data_ptr(), _lib.ptr(xin), n,
                  ctypes.addressof(c), o, order, newest, PRED[prediction_type], int(cfg),
                  float(guidance or 0.0), float(sigma), float(in_scale or 0.0), _lib.stream())
        return
    lms_step_reference(eps, x, ring, coefs, newest, sigma, guidance, prediction_type, in_scale, xin)


def lms_step_reference(eps, x, ring, coefs, newest, sigma, guidance, prediction_type="epsilon", in_scale=None,
                       xin=None):
    order = ring.shape[0]
    e = eps.float()
    if guidance is not None:
        eu, ec = e.chunk(2)
        e = eu + guidance * (ec - eu)
    s = float(sigma)
    if prediction_type == "epsilon":
        x0 = x - s * e
    elif prediction_type == "v_prediction":
        x0 = e * (-s / (s ** 2 + 1) ** 0.5) + x / (s ** 2 + 1)
    else:
        x0 = e
    d = (x - x0) / s
    ring[newest].view_as(d).copy_(d)
    acc = torch.zeros_like(x)
    for j, c in enumerate(coefs):
        acc = acc + c * ring[(newest - j) % order].view_as(x)
    x.add_(acc)
    if xin is not None:
        v = (x * in_scale).to(xin.dtype)
        if guidance is not None:
            xin.copy_(torch.cat([v, v]))
        else:
            xin.copy_(v)


__all__ = ["lms_step", "lms_step_reference", "PRED"]
