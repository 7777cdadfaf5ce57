"""Logits processing + sampling (K11/K31/K32), HF ``generate`` semantics.

The reference samples with HF ``generate`` (finetuner-workflow/finetuner/
finetuner.py:861-875: top_k 50, top_p .95, temperature 1.0, repetition
penalty 1.1, bad_words = [[eos]]; evaluator.py:201-213; bloom.py:68-77) and
with FasterTransformer's runtime_top_k / runtime_top_p / temperature /
repetition_penalty / bad_words_list / stop_words_list / is_return_log_probs
(download-weights-job-gptj.yml:101-175). One function covers both.

On GPU (bf16/fp32 logits) the whole chain -- penalty + bans + temperature +
top-k threshold + top-p nucleus + Philox multinomial + log-prob of the chosen
token -- runs in ``kca_sample_logits`` (csrc/kernels/decode.hip). Greedy rows,
top-k rows (k <= 64) and top-p-only rows of bf16 logits take the multi-workgroup
sampler: each row split over 16 chunk workgroups (32 for vocabularies past 50k,
BLOOM's 250,880) that publish their chunk maxima / normalisers / candidate lists,
the last one to arrive merging them; a top-p-only row whose candidates do not
hold the nucleus is marked and re-sampled by the one-workgroup register kernel
launched after it, which also takes every other row (top_k > 64, pure
multinomial, fp32 logits). The choice is made per row on the device, so captured
decode graphs serve any mix of request parameters. The torch path below is the
reference semantics.
"""
from __future__ import annotations

import torch

from ..ops import _lib


def apply_repetition_penalty(logits: torch.Tensor, seen: torch.Tensor, penalty: float):
    """HF RepetitionPenaltyLogitsProcessor: for ids already in the sequence,
    score / p if score > 0 else score * p. ``seen``: [B, T] token ids."""
    if penalty == 1.0 or seen is None or seen.numel() == 0:
        return logits
    sc = torch.gather(logits, 1, seen)
    sc = torch.where(sc < 0, sc * penalty, sc / penalty)
    return logits.scatter(1, seen, sc)


def top_k_top_p_filter(logits: torch.Tensor, top_k: int = 0, top_p: float = 1.0,
                       min_keep: int = 1) -> torch.Tensor:
    if top_k and top_k > 0:
        k = min(max(top_k, min_keep), logits.shape[-1])
        kth = torch.topk(logits, k, dim=-1).values[..., -1:]
        logits = logits.masked_fill(logits < kth, float("-inf"))
    if top_p is not None and top_p < 1.0:
        srt, idx = torch.sort(logits, descending=False, dim=-1)
        cum = srt.softmax(-1).cumsum(-1)
        remove = cum <= (1 - top_p)
        remove[..., -min_keep:] = False
        mask = remove.scatter(1, idx, remove)
        logits = logits.masked_fill(mask, float("-inf"))
    return logits


def sample_next(logits: torch.Tensor, *, seen: torch.Tensor | None = None, do_sample: bool = True,
                temperature: float = 1.0, top_k: int = 0, top_p: float = 1.0,
                repetition_penalty: float = 1.0, bad_words_ids=None, generator=None,
                return_logprobs: bool = False):
    """logits [B, V] -> next ids [B] (+ log-prob of the chosen id, from the
    distribution after penalties and temperature, like FT's output_log_probs)."""
    x = logits.float()
    x = apply_repetition_penalty(x, seen, repetition_penalty)
    if bad_words_ids:
        single = [w[0] for w in bad_words_ids if len(w) == 1]
        if single:
            x[:, single] = float("-inf")
        multi = [w for w in bad_words_ids if len(w) > 1]
        if multi and seen is not None:
            for w in multi:  # ban the last token of a multi-token bad word if its prefix just occurred
                pre = torch.tensor(w[:-1], device=seen.device)
                if seen.shape[1] >= len(pre):
                    hit = (seen[:, -len(pre):] == pre).all(-1)
                    x[hit, w[-1]] = float("-inf")
    if do_sample and temperature and temperature != 1.0:
        x = x / temperature
    logp_full = torch.log_softmax(x, dim=-1) if return_logprobs else None
    if do_sample:
        x = top_k_top_p_filter(x, top_k, top_p)
        probs = torch.softmax(x, dim=-1)
        nxt = torch.multinomial(probs, 1, generator=generator).squeeze(-1)
    else:
        nxt = torch.argmax(x, dim=-1)
    if return_logprobs:
        return nxt, logp_full.gather(1, nxt[:, None]).squeeze(-1)
    return nxt
