"""GPT-J parallel block with its elementwise work folded into the GEMM operand passes.

GPT-J (and only GPT-J among the reference's models: shared LayerNorm +
parallel residual, finetuner-workflow/finetuner/finetuner.py:789-831 loads it
through HF ``GPTJForCausalLM``) computes ``h + attn(ln(h)) + mlp(ln(h))``.
The four block GEMMs stay separate hipBLASLt calls in the TN layout
(ops/linear.py; concatenating [Wqkv; Wfc_in] and [Wout | Wfc_out] into two
bigger GEMMs measured 3 % slower in the training step on MI355X -- the
stand-alone 3-4.5 % win of bench/gemm_accum_bench.py does not survive in
context), and everything between them is fused into the passes the TN
weight-gradient GEMMs need anyway (csrc/kernels/block_fusion.hip):

  forward   qkv = x Wqkv^T, u = x Wfc_in^T + b (RoPE in place, flash attention)
            ``kca_gelu_fwd_t``: g = gelu(u) AND g^T (saved instead of g, so
            the backward never transposes the 16384-wide activation)
            a = o Wout^T, m = g Wfc_out^T + b2 (both go into the next
            LayerNorm's fused residual add)
  backward  da == dm (one residual grad): ONE ``kca_transpose_colsum`` gives
            dm^T and the fc_out bias grad for both dW GEMMs
            ``kca_gelu_bwd_t``: du = dg * gelu'(u), du^T and the fc_in bias
            partial sums in one pass
            dx = dqkv Wqkv + du Wfc_in accumulated in place (no autograd add)
            x^T transposed once for both input-side dW GEMMs

Weight gradients go to the parameter's gradient sink (ops/grad_sink.py) when
the training engine registered one (straight into its fp32 accumulation
buffer), otherwise back to autograd. Transposed weight copies are the block
TLinears' own ``weight_t`` (refreshed by the engine after every step).
"""
from __future__ import annotations

import torch
import torch.nn.functional as F

from . import _lib, grad_sink
from .attention import _bwd as _attn_bwd
from .attention import _fwd as _attn_fwd
from .attention import native_mask
from .linear import transpose
from .rope import apply_rotary_


def eligible(cfg) -> bool:
    """Block shapes/features the fused path implements (GPT-J family)."""
    d, f = cfg.hidden, cfg.ffn_dim
    return (cfg.parallel_residual and cfg.shared_ln and cfg.rotary_dim > 0 and not cfg.qkv_bias
            and not cfg.out_bias and not cfg.alibi and not cfg.attention_layers
            and d % 64 == 0 and f % 64 == 0 and cfg.head_dim in (64, 128, 256))


class FusedParallelBlock:
    """Fused training path of one GPT-J block (uses the TLinears' weight_t)."""

    def __init__(self, blk):
        self.blk = blk
        self.tanh = blk.mlp.approx == "tanh"

    def refresh(self):  # the TLinears own the transposed copies
        pass

    def applies(self, x: torch.Tensor, kv_len=None) -> bool:
        a, m = self.blk.attn, self.blk.mlp
        return (x.is_cuda and x.dtype == torch.bfloat16 and x.dim() == 3 and x.is_contiguous()
                and (x.shape[0] * x.shape[1]) % 64 == 0
                and all(t.weight_t is not None for t in (a.qkv, a.out, m.fc_in, m.fc_out)))

    def __call__(self, x: torch.Tensor, kv_len=None):
        attn, mlp = self.blk.attn, self.blk.mlp
        return _FusedBlockFn.apply(x, attn.qkv.weight, attn.out.weight, mlp.fc_in.weight, mlp.fc_in.bias,
                                   mlp.fc_out.weight, mlp.fc_out.bias, self, native_mask(kv_len, x.device))


def _col_sums(part: torch.Tensor, dtype) -> torch.Tensor:
    out = torch.empty(part.shape[1], device=part.device, dtype=dtype)
    _lib.call("kca_col_reduce_f32", part.data_ptr(), part.shape[0], part.shape[1], out.data_ptr(), None,
              _lib.stream())
    return out


def _emit(param: torch.Tensor, grad: torch.Tensor):
    """Hand a weight gradient to the engine's sink (returns None) or back to autograd."""
    if param is None or grad is None or not param.requires_grad:
        return None
    sink = grad_sink.lookup(param)
    if sink is not None:
        sink(param, grad)
        return None
    return grad


def _emit_wgrad(param: torch.Tensor, a: torch.Tensor, w: torch.Tensor):
    """Weight gradient ``a w^T`` (TN operands), handed on like ``_emit``."""
    if param is None or not param.requires_grad:
        return None
    return _emit(param, F.linear(a, w))


class _FusedBlockFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w_qkv, w_out, w_fc_in, b_fc_in, w_fc_out, b_fc_out, fb, kv_len):
        blk = fb.blk
        cfg = blk.cfg
        a = blk.attn
        B, S, d = x.shape
        T = B * S
        H, D = a.n_heads, a.head_dim
        x2 = x.reshape(T, d)
        qkv = F.linear(x2, w_qkv)  # [T, 3d]
        u = F.linear(x2, w_fc_in, b_fc_in)  # [T, f]
        f = u.shape[1]
        q5 = qkv.view(B, S, 3, H, D)
        q, k, v = q5[:, :, 0], q5[:, :, 1], q5[:, :, 2]
        apply_rotary_(q, k, cfg.rotary_dim, S, cfg.rotary_interleaved, cfg.rotary_base, 1.0)
        o, lse = _attn_fwd(q, k, v, True, a.scale, kv_len, None)
        o = o.view(T, d)
        g = torch.empty_like(u)
        gt = torch.empty(f, T, device=x.device, dtype=x.dtype)
        _lib.call("kca_gelu_fwd_t", u.data_ptr(), f, g.data_ptr(), f, gt.data_ptr(), T, T, f, int(fb.tanh),
                  _lib.stream())
        out_a = F.linear(o, w_out)
        out_m = F.linear(g, w_fc_out, b_fc_out)
        ctx.save_for_backward(x, qkv, u, o, gt, lse, kv_len)
        ctx.fb = fb
        return out_a.view(B, S, d), out_m.view(B, S, d)

    @staticmethod
    def backward(ctx, da, dm):
        x, qkv, u, o, gt, lse, kv_len = ctx.saved_tensors
        fb = ctx.fb
        blk = fb.blk
        cfg = blk.cfg
        a, mlp = blk.attn, blk.mlp
        B, S, d = x.shape
        T, f = B * S, u.shape[1]
        H, D = a.n_heads, a.head_dim
        dev, dt = x.device, x.dtype
        st = _lib.stream()
        dm2 = dm.reshape(T, d).contiguous() if dm is not None else torch.zeros(T, d, device=dev, dtype=dt)
        da2 = da.reshape(T, d).contiguous() if da is not None else torch.zeros(T, d, device=dev, dtype=dt)

        # ---- output projections: dm^T (+ fc_out bias grad) once, shared with da when da is dm
        dmt = torch.empty(d, T, device=dev, dtype=dt)
        part = torch.empty(T // 64, d, device=dev, dtype=torch.float32) if b_needed(mlp.fc_out) else None
        _lib.call("kca_transpose_colsum", dm2.data_ptr(), d, dmt.data_ptr(), T, _lib.ptr(part), T, d, st)
        g_b_out = _emit(mlp.fc_out.bias, _col_sums(part, dt)) if part is not None else None
        dg = F.linear(dm2, mlp.fc_out.weight_t)  # [T, f]
        g_fc_out = _emit_wgrad(mlp.fc_out.weight, dmt, gt)
        if da2.data_ptr() != dm2.data_ptr():
            dat = transpose(da2)
        else:
            dat = dmt
        g_out = _emit_wgrad(a.out.weight, dat, transpose(o))
        do = F.linear(da2, a.out.weight_t).view(B, S, H, D)
        del dat, dmt

        # ---- attention backward (+ RoPE transpose) into dqkv
        q5 = qkv.view(B, S, 3, H, D)
        dqkv = torch.empty_like(qkv)
        d5 = dqkv.view(B, S, 3, H, D)
        dq, dk, dv = d5[:, :, 0], d5[:, :, 1], d5[:, :, 2]
        _attn_bwd(q5[:, :, 0], q5[:, :, 1], q5[:, :, 2], o.view(B, S, H, D), do, lse, dq, dk, dv, True,
                  a.scale, kv_len, None)
        apply_rotary_(dq, dk, cfg.rotary_dim, S, cfg.rotary_interleaved, cfg.rotary_base, -1.0)
        del do

        # ---- GELU backward: du, du^T, fc_in bias partials in one pass
        du = torch.empty_like(u)
        dut = torch.empty(f, T, device=dev, dtype=dt)
        part = torch.empty(T // 64, f, device=dev, dtype=torch.float32) if b_needed(mlp.fc_in) else None
        _lib.call("kca_gelu_bwd_t", dg.data_ptr(), f, u.data_ptr(), f, du.data_ptr(), f, dut.data_ptr(), T,
                  _lib.ptr(part), T, f, int(fb.tanh), st)
        del dg
        g_b_in = _emit(mlp.fc_in.bias, _col_sums(part, dt)) if part is not None else None

        # ---- input side: dx = dqkv Wqkv + du Wfc_in (accumulated in place), x^T once
        dx = None
        if ctx.needs_input_grad[0]:
            dx = F.linear(dqkv, a.qkv.weight_t)
            dx.addmm_(du, mlp.fc_in.weight_t.t())
        xt = transpose(x.reshape(T, d))
        g_fc_in = _emit_wgrad(mlp.fc_in.weight, dut, xt)
        del dut, du
        g_qkv = _emit_wgrad(a.qkv.weight, transpose(dqkv), xt)
        return (dx.view(B, S, d) if dx is not None else None, g_qkv, g_out, g_fc_in, g_b_in, g_fc_out, g_b_out,
                None, None)


def b_needed(lin) -> bool:
    return lin.bias is not None and lin.bias.requires_grad


__all__ = ["FusedParallelBlock", "eligible"]
