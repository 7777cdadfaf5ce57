"""Fused cross-entropy with ignore_index (K6) and fp32 MSE (K19)."""
from __future__ import annotations

import torch
import torch.nn.functional as F

from . import _lib


class _CrossEntropyFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, logits, labels, ignore_index, inplace_grad):
        n, V = logits.shape
        if logits.stride(1) != 1:
            logits = logits.contiguous()
        labels = labels.contiguous().to(torch.int64)
        loss = torch.empty(n, device=logits.device, dtype=torch.float32)
        lse = torch.empty_like(loss)
        _lib.call("kca_cross_entropy_fwd", logits.data_ptr(), logits.stride(0), labels.data_ptr(),
                  n, V, ignore_index, loss.data_ptr(), lse.data_ptr(), _lib.stream())
        ctx.save_for_backward(logits, labels, lse)
        ctx.ignore_index = ignore_index
        ctx.inplace = inplace_grad
        return loss

    @staticmethod
    def backward(ctx, dloss):
        logits, labels, lse = ctx.saved_tensors
        n, V = logits.shape
        dl = logits if ctx.inplace else torch.empty_like(logits)
        dloss = dloss.contiguous().float()
        _lib.call("kca_cross_entropy_bwd", logits.data_ptr(), logits.stride(0), labels.data_ptr(),
                  lse.data_ptr(), dloss.data_ptr(), 1.0, n, V, ctx.ignore_index, dl.data_ptr(),
                  dl.stride(0), _lib.stream())
        return dl, None, None, None


def cross_entropy(logits: torch.Tensor, labels: torch.Tensor, ignore_index: int = -100,
                  reduction: str = "mean", inplace_grad: bool = True) -> torch.Tensor:
    """Token-level CE over ``logits [N, V]`` (bf16) with HF semantics: mean over
    non-ignored tokens. ``inplace_grad`` lets the backward overwrite the logits
    buffer with dlogits (saves an N x V allocation; the logits must not be
    needed afterwards)."""
    if _lib.use_native(logits):
        per_tok = _CrossEntropyFn.apply(logits, labels, ignore_index, inplace_grad)
    else:
        per_tok = F.cross_entropy(logits.float(), labels, ignore_index=ignore_index,
                                  reduction="none")
    if reduction == "none":
        return per_tok
    if reduction == "sum":
        return per_tok.sum()
    valid = (labels != ignore_index).sum().clamp_min(1)
    return per_tok.sum() / valid


def mse_loss(pred: torch.Tensor, target: torch.Tensor, reduction: str = "mean") -> torch.Tensor:
    """fp32 MSE as the SD trainer computes it (sd-finetuner/finetuner.py:513-529)."""
    return F.mse_loss(pred.float(), target.float(), reduction=reduction)
