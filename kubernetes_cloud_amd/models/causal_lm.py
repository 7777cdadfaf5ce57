"""Native decoder-only LM covering GPT-2, GPT-Neo(X)/Pythia, GPT-J, BLOOM and
XGLM / fairseq-dense (scaled embeddings + fixed sinusoidal positions, pre-LN).

What the reference runs through HF ``AutoModelForCausalLM`` + DeepSpeed
(finetuner-workflow/finetuner/finetuner.py:789-831 load, 469-493 loss) and the
FT / DS-Inference engines (online-inference/fastertransformer, bloom-176b-*),
built the MI355X way:

* one fused QKV projection per layer (hipBLASLt GEMM), RoPE applied in place on
  its output and flash attention reading Q/K/V straight from that buffer
  (``ops.qkv_rope_attention``) -- the backward produces one fused dQKV buffer;
* every residual add is fused into the *next* LayerNorm (``ops.layer_norm``
  with ``residual=``), so the residual stream is written once per sub-layer;
* bias+GELU: the bias rides in the GEMM epilogue (addmm), GELU is a 16-B/lane
  HIP kernel; the LM-head cross-entropy never materialises fp32 logits.

The forward carries ``(h, pending)`` between blocks: ``pending`` are the branch
outputs not yet added to the residual stream ``h``.
"""
from __future__ import annotations

import math

import torch
import torch.nn as nn
import torch.nn.functional as F
from torch.utils.checkpoint import checkpoint

from .. import ops
from ..ops.linear import TLinear
from .config import LMConfig


def alibi_slopes(n_heads: int) -> torch.Tensor:
    """BLOOM / Press et al. ALiBi head slopes (closest power of two + interleave)."""
    def pow2(n):
        start = 2 ** (-(2 ** -(math.log2(n) - 3)))
        return [start * (start ** i) for i in range(n)]
    if math.log2(n_heads).is_integer():
        s = pow2(n_heads)
    else:
        c = 2 ** math.floor(math.log2(n_heads))
        s = pow2(c) + pow2(2 * c)[0::2][: n_heads - c]
    return torch.tensor(s, dtype=torch.float32)


def mask_to_kv(mask: torch.Tensor):
    """HF attention_mask [B, S] (1 = real token) -> what the attention kernels take:

    * ``None``            every token attends (no mask work at all);
    * int32 [B] lengths   right padding (each row a prefix of ones);
    * bool [B, S]         a mask with holes, e.g. the interior EOS separators of
                          the last context of a pad == eos dataset
                          (finetuner.py:674-691) -- exact HF semantics; the
                          kernels take it as a packed key bitmap.

    A host mask is classified exactly. A device mask is never read back (no
    host sync): it is taken as right padding, length = last real token + 1."""
    if mask.device.type != "cpu":
        S = mask.shape[-1]
        pos = torch.arange(1, S + 1, device=mask.device, dtype=torch.int32)
        return (mask.to(torch.int32) * pos).amax(-1).to(torch.int32)
    m = mask.bool()
    if bool(m.all()):
        return None
    pos = torch.arange(1, m.shape[-1] + 1, dtype=torch.int64)
    last = (m.long() * pos).amax(-1)
    if bool((m.long().sum(-1) == last).all()):
        return last.to(torch.int32)
    return m


class SinusoidalPositions(nn.Module):
    """fairseq / XGLM fixed positions: row p + offset of the tensor2tensor table
    [sin(p w_i) | cos(p w_i)], w_i = 10000^(-i / (d/2 - 1)). Computed on the fly
    in fp32 (no parameters, nothing to load or shard)."""

    def __init__(self, d: int, offset: int):
        super().__init__()
        self.d, self.offset = d, offset

    def forward(self, pos: torch.Tensor) -> torch.Tensor:
        half = self.d // 2
        w = torch.exp(torch.arange(half, device=pos.device, dtype=torch.float32) * -(math.log(10000.0) / (half - 1)))
        a = (pos.to(torch.float32) + self.offset).unsqueeze(-1) * w
        e = torch.cat([torch.sin(a), torch.cos(a)], dim=-1)
        if self.d % 2:
            e = F.pad(e, (0, 1))
        return e


class LayerNorm(nn.Module):
    def __init__(self, d: int, eps: float):
        super().__init__()
        self.weight = nn.Parameter(torch.ones(d))
        self.bias = nn.Parameter(torch.zeros(d))
        self.eps = eps

    def forward(self, x, residual=()):
        return ops.layer_norm(x, self.weight, self.bias, self.eps, residual=residual)


class Attention(nn.Module):
    def __init__(self, cfg: LMConfig, layer_idx: int):
        super().__init__()
        d = cfg.hidden
        self.cfg = cfg
        self.n_heads = cfg.n_heads
        self.head_dim = cfg.head_dim
        self.qkv = TLinear(d, 3 * d, bias=cfg.qkv_bias)
        self.out = TLinear(d, d, bias=cfg.out_bias)
        self.window = 0
        if cfg.attention_layers and cfg.attention_layers[layer_idx] == "local":
            self.window = cfg.local_window
        self.scale = cfg.attn_scale if cfg.attn_scale is not None else 1.0 / math.sqrt(self.head_dim)
        if cfg.alibi:
            self.register_buffer("alibi", alibi_slopes(cfg.n_heads), persistent=False)
        else:
            self.alibi = None

    def forward(self, x: torch.Tensor, kv_len: torch.Tensor | None = None) -> torch.Tensor:
        B, S, _ = x.shape
        qkv = self.qkv(x)
        cfg = self.cfg
        if cfg.rotary_dim > 0:
            o = ops.qkv_rope_attention(qkv, self.n_heads, self.head_dim, cfg.rotary_dim,
                                       cfg.rotary_interleaved, causal=True, base=cfg.rotary_base,
                                       scale=self.scale, kv_len=kv_len)
        else:
            # (GPT-Neo local layers: the kernels skip the tiles left of the band, ``window``)
            v5 = qkv.view(B, S, 3, self.n_heads, self.head_dim)
            o = ops.flash_attention(v5[:, :, 0], v5[:, :, 1], v5[:, :, 2], causal=True,
                                    scale=self.scale, kv_len=kv_len, alibi=self.alibi, window=self.window)
            o = o.reshape(B, S, -1)
        return self.out(o)


class MLP(nn.Module):
    def __init__(self, cfg: LMConfig):
        super().__init__()
        self.fc_in = TLinear(cfg.hidden, cfg.ffn_dim, bias=cfg.mlp_bias)
        self.fc_out = TLinear(cfg.ffn_dim, cfg.hidden, bias=cfg.mlp_bias)
        self.approx = cfg.gelu_approx

    def forward(self, x):
        return self.fc_out(ops.gelu(self.fc_in(x), self.approx))


class Block(nn.Module):
    def __init__(self, cfg: LMConfig, layer_idx: int):
        super().__init__()
        self.cfg = cfg
        self.ln_1 = LayerNorm(cfg.hidden, cfg.ln_eps)
        self.attn = Attention(cfg, layer_idx)
        self.ln_2 = None if cfg.shared_ln else LayerNorm(cfg.hidden, cfg.ln_eps)
        self.mlp = MLP(cfg)
        self.fused = None  # ops.fused_block.FusedParallelBlock (GPT-J training path)

    def forward(self, h, kv_len, *pending):
        if pending:
            x, h = self.ln_1(h, residual=pending)
        else:
            x = self.ln_1(h)
        if self.fused is not None and torch.is_grad_enabled() and self.fused.applies(x, kv_len):
            a, m = self.fused(x, kv_len)
            return h, a, m
        if self.cfg.parallel_residual:
            a = self.attn(x, kv_len)
            x2 = x if self.ln_2 is None else self.ln_2(h)
            m = self.mlp(x2)
            return h, a, m
        a = self.attn(x, kv_len)
        x2, h = self.ln_2(h, residual=(a,))
        m = self.mlp(x2)
        return h, m


class CausalLM(nn.Module):
    def __init__(self, cfg: LMConfig):
        super().__init__()
        self.cfg = cfg
        d = cfg.hidden
        self.wte = nn.Embedding(cfg.vocab_size, d)
        if cfg.sinusoidal_pos:
            self.wpe = SinusoidalPositions(d, cfg.pos_offset)
        else:
            self.wpe = nn.Embedding(cfg.max_pos, d) if cfg.learned_pos else None
        self.emb_ln = LayerNorm(d, cfg.ln_eps) if cfg.embed_ln else None
        self.h = nn.ModuleList([Block(cfg, i) for i in range(cfg.n_layers)])
        self.ln_f = LayerNorm(d, cfg.ln_eps)
        if cfg.tie_embeddings:
            self.lm_head = None
        else:
            # TLinear: dX of the LM head as a TN GEMM off a transposed weight copy (the NN dgrad ran at
            # ~1.1 PF/s, 12 ms of the GPT-J step: profiles/gptj_step_kernel_stats_r4.md)
            self.lm_head = TLinear(d, cfg.vocab_size, bias=cfg.lm_head_bias)
        self.gradient_checkpointing = False

    # ------------------------------------------------------------------ init
    @torch.no_grad()
    def init_weights(self, std: float = 0.02, seed: int | None = None):
        g = torch.Generator(device="cpu")
        gd = None
        if seed is not None:
            g.manual_seed(seed)
        for name, p in self.named_parameters():
            if p.dim() >= 2:
                if p.is_cuda:
                    # seeded device generator: every DP rank builds identical weights
                    if gd is None:
                        gd = torch.Generator(device=p.device)
                        if seed is not None:
                            gd.manual_seed(seed)
                        else:
                            gd.seed()
                    p.normal_(0.0, std, generator=gd)
                else:
                    p.copy_(torch.randn(p.shape, generator=g) * std)
            elif name.endswith("weight"):
                p.fill_(1.0)
            else:
                p.zero_()
        return self

    # train/engine.py: ZeRO-1/2 parameter all-gathers may finish under the next forward -- every
    # parameter is read inside a ModuleList block's forward or by a module called for it (wte, ln_f,
    # lm_head; the tied head reads wte after the embedding's pre-hook)
    supports_deferred_param_gather = True

    def enable_tn_grads(self, on: bool = True):
        """TN-layout backward GEMMs for the block linears (ops/linear.py): keeps a
        transposed bf16 copy of each block weight (+1x the block weights in HBM).
        GPT-J-shaped blocks additionally run their training forward/backward
        through ops/fused_block.py (GELU, bias grads and operand transposes
        folded into single passes; KCA_FUSED_BLOCK=0 keeps the per-module
        autograd path)."""
        import os

        from ..ops import fused_block
        fuse = (on and os.environ.get("KCA_FUSED_BLOCK", "1") not in ("0", "false")
                and fused_block.eligible(self.cfg))
        for blk in self.h:
            w = blk.attn.qkv.weight
            blk.fused = None
            if fuse and w.is_cuda and w.dtype == torch.bfloat16:
                blk.fused = fused_block.FusedParallelBlock(blk)
        for m in self.modules():
            if isinstance(m, TLinear):
                m.enable_tn(on)

    @torch.no_grad()
    def refresh_transposed_weights(self):
        """Re-derive the transposed / concatenated weight copies after the weights changed."""
        for m in self.modules():
            if isinstance(m, TLinear):
                m.refresh_transposed()
        for blk in self.h:
            if blk.fused is not None:
                blk.fused.refresh()

    def gradient_checkpointing_enable(self, on: bool = True):
        self.gradient_checkpointing = on

    def resize_token_embeddings(self, n: int):
        """HF resize_token_embeddings (finetuner.py:885): grow/shrink vocab rows."""
        old = self.wte.weight
        if n == old.shape[0]:
            return
        new = nn.Embedding(n, old.shape[1]).to(old.device, old.dtype)
        with torch.no_grad():
            new.weight.normal_(0.0, 0.02)
            k = min(n, old.shape[0])
            new.weight[:k] = old[:k]
        self.wte = new
        if self.lm_head is not None:
            oh = self.lm_head
            nh = TLinear(oh.in_features, n, bias=oh.bias is not None).to(old.device, old.dtype)
            with torch.no_grad():
                nh.weight.normal_(0.0, 0.02)
                nh.weight[:k] = oh.weight[:k]
                if oh.bias is not None:
                    nh.bias.zero_()
                    nh.bias[:k] = oh.bias[:k]
            self.lm_head = nh
        self.cfg.vocab_size = n

    # --------------------------------------------------------------- forward
    def embed(self, input_ids: torch.Tensor, pos: torch.Tensor | None = None) -> torch.Tensor:
        """Token (+ position) embeddings (+ BLOOM's embedding LayerNorm); ``pos``
        defaults to 0..S-1 (the training forward, a fresh prefill)."""
        h = self.wte(input_ids)
        if self.cfg.embed_scale != 1.0:
            h = h * self.cfg.embed_scale
        if self.wpe is not None:
            if pos is None:
                pos = torch.arange(input_ids.shape[-1], device=input_ids.device)
            h = h + self.wpe(pos).to(h.dtype)
        if self.emb_ln is not None:
            h = self.emb_ln(h)
        return h

    def hidden_states(self, input_ids: torch.Tensor, attention_mask: torch.Tensor | None = None,
                      position_ids: torch.Tensor | None = None, kv_len: torch.Tensor | None = None):
        h = self.embed(input_ids, position_ids)
        if kv_len is None and attention_mask is not None:
            kv_len = mask_to_kv(attention_mask)
        if kv_len is not None:
            kv_len = kv_len.to(h.device, non_blocking=True)
        pending = ()
        for blk in self.h:
            if self.gradient_checkpointing and self.training and torch.is_grad_enabled():
                out = checkpoint(blk, h, kv_len, *pending, use_reentrant=False)
            else:
                out = blk(h, kv_len, *pending)
            h, pending = out[0], tuple(out[1:])
        y, _ = self.ln_f(h, residual=pending) if pending else (self.ln_f(h), None)
        return y

    def logits_from_hidden(self, y: torch.Tensor) -> torch.Tensor:
        if self.lm_head is None:
            if getattr(self, "_param_linear", False):  # ZeRO-3 (train/engine.py)
                from ..ops.linear import param_linear
                return param_linear(y, self.wte.weight)
            return F.linear(y, self.wte.weight)
        return self.lm_head(y)

    def forward(self, input_ids: torch.Tensor, attention_mask: torch.Tensor | None = None,
                labels: torch.Tensor | None = None, position_ids: torch.Tensor | None = None,
                kv_len: torch.Tensor | None = None):
        """``kv_len``: precomputed ``mask_to_kv(attention_mask)`` (the data
        collator does it on the host, so the forward never syncs)."""
        y = self.hidden_states(input_ids, attention_mask, position_ids, kv_len)
        logits = self.logits_from_hidden(y)
        if labels is None:
            return logits
        B, S = labels.shape
        shifted = torch.full_like(labels, -100)
        shifted[:, :-1] = labels[:, 1:]
        return ops.cross_entropy(logits.view(B * S, -1), shifted.view(-1), ignore_index=-100)

    def num_parameters(self) -> int:
        return sum(p.numel() for p in self.parameters())


def build_model(cfg: LMConfig, device="cpu", dtype=torch.bfloat16, seed: int | None = 0) -> CausalLM:
    with torch.device("meta"):
        m = CausalLM(cfg)
    m = m.to_empty(device=device).to(dtype)
    if cfg.alibi:
        for blk in m.h:
            blk.attn.alibi = alibi_slopes(cfg.n_heads).to(device)
    m.init_weights(seed=seed)
    return m
