"""Autoregressive generation over the native KV cache.

Serves the finetuner's periodic sampler (finetuner.py:538-630, 835-881), the
evaluator CLI (evaluator.py:175-219), the completion server (inference.py
80-96) and the KServe predictors (bloom.py:57-77, kserve_api.py:47-72).
Prefill runs the whole prompt through the flash-attention kernel in one pass;
each decode step appends one token per sequence to the cache (bottom-right
aligned causal attention over [0, start+1)).
"""
from __future__ import annotations

import dataclasses

import torch

from .sampling import sample_next


@dataclasses.dataclass
class GenerationConfig:
    max_new_tokens: int = 50
    min_new_tokens: int = 0
    do_sample: bool = True
    temperature: float = 1.0
    top_k: int = 50
    top_p: float = 1.0
    repetition_penalty: float = 1.0
    num_return_sequences: int = 1
    eos_token_id: int | None = None
    pad_token_id: int | None = None
    bad_words_ids: list | None = None
    stop_sequences: list | None = None  # list of token-id lists
    seed: int | None = None
    return_logprobs: bool = False


@dataclasses.dataclass
class GenerationResult:
    sequences: torch.Tensor        # [N, prompt + new] (padded with pad id after EOS)
    lengths: torch.Tensor          # [N] total valid length
    logprobs: torch.Tensor | None  # [N, new]
    prompt_len: int


@torch.no_grad()
def generate(model, input_ids: torch.Tensor, cfg: GenerationConfig) -> GenerationResult:
    """``input_ids``: [B, T] prompts of equal length (one request's samples)."""
    model.eval()
    dev = next(model.parameters()).device
    ids = input_ids.to(dev)
    if cfg.num_return_sequences > 1:
        ids = ids.repeat_interleave(cfg.num_return_sequences, 0)
    N, T = ids.shape
    total = T + cfg.max_new_tokens
    cache = model.new_cache(N, total)
    gen = None
    if cfg.seed is not None:
        gen = torch.Generator(device=dev)
        gen.manual_seed(cfg.seed)
    out = torch.empty(N, total, dtype=torch.long, device=dev)
    out[:, :T] = ids
    lps = torch.zeros(N, cfg.max_new_tokens, device=dev) if cfg.return_logprobs else None
    done = torch.zeros(N, dtype=torch.bool, device=dev)
    lengths = torch.full((N,), total, dtype=torch.long, device=dev)
    pad = cfg.pad_token_id if cfg.pad_token_id is not None else (cfg.eos_token_id or 0)
    logits = model.forward_cached(ids, cache, 0)
    for i in range(cfg.max_new_tokens):
        bad = cfg.bad_words_ids
        if cfg.eos_token_id is not None and i < cfg.min_new_tokens:
            bad = list(bad or []) + [[cfg.eos_token_id]]
        res = sample_next(logits, seen=out[:, :T + i], do_sample=cfg.do_sample,
                          temperature=cfg.temperature, top_k=cfg.top_k, top_p=cfg.top_p,
                          repetition_penalty=cfg.repetition_penalty, bad_words_ids=bad,
                          generator=gen, return_logprobs=cfg.return_logprobs)
        nxt, lp = (res if cfg.return_logprobs else (res, None))
        nxt = torch.where(done, torch.full_like(nxt, pad), nxt)
        out[:, T + i] = nxt
        if lp is not None:
            lps[:, i] = torch.where(done, torch.zeros_like(lp), lp)
        newly = ~done & _stopped(out, T + i + 1, nxt, cfg)
        lengths = torch.where(newly, torch.full_like(lengths, T + i + 1), lengths)
        done = done | newly
        if i + 1 == cfg.max_new_tokens or bool(done.all()):
            if bool(done.all()):
                out = out[:, :T + i + 1]
                if lps is not None:
                    lps = lps[:, :i + 1]
            break
        logits = model.forward_cached(nxt[:, None], cache, T + i)
    lengths = lengths.clamp(max=out.shape[1])
    return GenerationResult(out, lengths, lps, T)


def _stopped(out, upto, nxt, cfg: GenerationConfig):
    stop = torch.zeros_like(nxt, dtype=torch.bool)
    if cfg.eos_token_id is not None:
        stop |= nxt == cfg.eos_token_id
    for seq in cfg.stop_sequences or []:
        L = len(seq)
        if L and upto >= L:
            tgt = torch.tensor(seq, device=out.device)
            stop |= (out[:, upto - L:upto] == tgt).all(-1)
    return stop
