"""Fused SD training-step elementwise ops (``csrc/kernels/sd_train.hip``,
SURVEY K18/K19/K20).

* ``noise_prep``: VAE moments -> latent sample x0 = (mean + exp(logvar/2) e) *
  scale, DDPM x_t = sqrt(a_t) x0 + sqrt(1 - a_t) n and the epsilon / v target,
  in one pass with both normal draws from in-kernel Philox.
* ``mse_split``: fp32 MSE with the DreamBooth prior-preservation split
  (instance half + w * class half) as one reduction, gradient as one pass.

The references below are the same math in torch (the CPU path, and the pins of
the kernels in ``tests/test_kernels_gpu.py``); the reference finetuner's form is
sd-finetuner/finetuner.py:480-529.
"""
from __future__ import annotations

import ctypes

import torch

from . import _lib


def _strides(t: torch.Tensor):
    return (ctypes.c_longlong * 4)(*t.stride())


def noise_prep(mean: torch.Tensor, logvar: torch.Tensor, acp: torch.Tensor, scale: float, v_pred: bool,
               seed: int = 0, e: torch.Tensor | None = None, n: torch.Tensor | None = None,
               channels_last: bool | None = None, sample_base: int = 0, sample_stride: int = 1):
    """mean / logvar: [B, C, H, W] views of the VAE moments; acp: [B] fp32
    alphas_cumprod of each sample's timestep. Returns (noisy, target) bf16 in
    the moments' memory format (or ``channels_last`` when given). ``e`` / ``n``
    (logical [B, C, H, W]) replace the internal draws (tests). Local sample b draws as global sample
    ``sample_base + b * sample_stride`` of the step (data-parallel ranks: the same noise per sample
    whatever the split)."""
    B, C, H, W = mean.shape
    if channels_last is None:
        channels_last = mean.is_contiguous(memory_format=torch.channels_last) or (
            mean.stride(1) == 1 and mean.dim() == 4)
    fmt = torch.channels_last if channels_last else torch.contiguous_format
    if mean.is_cuda and mean.dtype == torch.bfloat16 and _lib.has("kca_sd_noise_prep"):
        assert logvar.stride() == mean.stride() and acp.dtype == torch.float32 and acp.is_contiguous()
        noisy = torch.empty(B, C, H, W, device=mean.device, dtype=torch.bfloat16, memory_format=fmt)
        target = torch.empty_like(noisy)
        ec = e.to(torch.bfloat16).contiguous() if e is not None else None
        nc = n.to(torch.bfloat16).contiguous() if n is not None else None
        assert acp.numel() == B and (ec is None or ec.shape == mean.shape) and (nc is None or nc.shape == mean.shape)
        s_in, s_out = _strides(mean), _strides(noisy)  # keep the host arrays alive across the call
        _lib.call("kca_sd_noise_prep", mean.data_ptr(), logvar.data_ptr(), ctypes.addressof(s_in),
                  noisy.data_ptr(), target.data_ptr(), ctypes.addressof(s_out), acp.data_ptr(),
                  _lib.ptr(ec), _lib.ptr(nc), B, C, H, W, float(scale), int(v_pred), seed & ((1 << 64) - 1),
                  int(sample_base), int(sample_stride), _lib.stream())
        return noisy, target
    return noise_prep_reference(mean, logvar, acp, scale, v_pred, e, n, fmt)


def noise_prep_reference(mean, logvar, acp, scale, v_pred, e=None, n=None, fmt=torch.contiguous_format):
    dt = mean.dtype
    if e is None:
        e = torch.randn(mean.shape, device=mean.device)
    if n is None:
        n = torch.randn(mean.shape, device=mean.device)
    std = torch.exp(0.5 * logvar.float().clamp(-30.0, 20.0))
    # DiagonalGaussian.sample() in the VAE dtype, then * scale (the reference's latents stay bf16)
    x0 = ((mean.float() + std * e.float()).to(dt).float() * scale).to(dt).float()
    nb = n.to(dt).float()
    a = acp.float().view(-1, 1, 1, 1).to(mean.device)
    noisy = (a.sqrt() * x0 + (1 - a).sqrt() * nb).to(dt)
    target = ((a.sqrt() * nb - (1 - a).sqrt() * x0) if v_pred else nb).to(dt)
    return noisy.contiguous(memory_format=fmt), target.contiguous(memory_format=fmt)


class _MSESplit(torch.autograd.Function):
    @staticmethod
    def forward(ctx, pred, target, split, w):
        n = pred.numel()
        loss = torch.empty((), device=pred.device, dtype=torch.float32)
        ws = torch.empty(1024, device=pred.device, dtype=torch.float32)
        _lib.call("kca_mse_split_fwd", pred.data_ptr(), target.data_ptr(), n, split, float(w), ws.data_ptr(),
                  ws.numel(), loss.data_ptr(), _lib.stream())
        ctx.save_for_backward(pred, target)
        ctx.split, ctx.w = split, w
        return loss

    @staticmethod
    def backward(ctx, g):
        pred, target = ctx.saved_tensors
        gp = torch.empty_like(pred)
        g = g.float().contiguous()
        _lib.call("kca_mse_split_bwd", pred.data_ptr(), target.data_ptr(), g.data_ptr(), pred.numel(), ctx.split,
                  float(ctx.w), gp.data_ptr(), _lib.stream())
        return gp, None, None, None


def mse_split(pred: torch.Tensor, target: torch.Tensor, prior_weight: float | None = None) -> torch.Tensor:
    """mean((pred - target)^2) in fp32; with ``prior_weight`` the batch halves are
    the instance and class (prior) examples: mse(first) + w * mse(second)."""
    split_batch = prior_weight is not None
    if (pred.is_cuda and pred.dtype == torch.bfloat16 and target.dtype == torch.bfloat16
            and pred.stride() == target.stride() and _lib.has("kca_mse_split_fwd")
            and (pred.is_contiguous() or pred.is_contiguous(memory_format=torch.channels_last))):
        n = pred.numel()
        split = n // 2 if split_batch else n
        return _MSESplit.apply(pred, target, split, float(prior_weight or 0.0))
    return mse_split_reference(pred, target, prior_weight)


def mse_split_reference(pred, target, prior_weight=None):
    import torch.nn.functional as F
    if prior_weight is None:
        return F.mse_loss(pred.float(), target.float())
    p_i, p_c = pred.chunk(2)
    t_i, t_c = target.chunk(2)
    return F.mse_loss(p_i.float(), t_i.float()) + prior_weight * F.mse_loss(p_c.float(), t_c.float())


__all__ = ["noise_prep", "noise_prep_reference", "mse_split", "mse_split_reference"]
