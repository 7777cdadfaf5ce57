"""Beam search on the slot KV cache (FasterTransformer's
``beam_width`` / ``len_penalty`` / ``beam_search_diversity_rate`` inputs,
online-inference/fastertransformer/download-weights-job-gptj.yml:115-163).

One request owns ``W`` cache slots. Each step scores all beams with one
decode pass (top-2W log-probs per beam on device), keeps the W best
continuations, moves ended hypotheses (end_id) to the finished pool with
length-normalised score ``logp / len ** len_penalty`` and re-orders the KV cache
rows of surviving beams to their parents (``ModelRunner.copy_slots``).
A diversity rate d penalises the r-th ranked candidate of a parent by ``d*r``
(FT's "diverse beam search" knob).
"""
from __future__ import annotations

import dataclasses

import torch


@dataclasses.dataclass
class BeamResult:
    sequences: list      # [n_return] token lists (generated part)
    scores: list         # length-normalised cumulative log-probs
    cum_logprobs: list   # raw cumulative log-probs


def beam_search(runner, prompt: list[int], slots: list[int], max_new_tokens: int, end_id: int | None = None,
                len_penalty: float = 1.0, diversity_rate: float = 0.0, n_return: int = 1) -> BeamResult:
    W = len(slots)
    T = len(prompt)
    logits = runner.prefill(torch.tensor([prompt]), [slots[0]])
    lp0 = torch.log_softmax(logits.float(), -1)[0]
    runner.copy_slots(slots[1:], [slots[0]] * (W - 1), T)
    kk = min(2 * W, lp0.shape[-1])
    top_lp, top_id = lp0.topk(kk)
    beams = []  # (cum_lp, tokens)
    finished = []
    for lp, t in zip(top_lp.tolist(), top_id.tolist()):
        if end_id is not None and t == end_id:
            finished.append((lp, [t]))
        elif len(beams) < W:
            beams.append((lp, [t]))
        if len(beams) == W:
            break
    step = 1
    while beams and step < max_new_tokens:
        n = len(beams)
        cur_slots = slots[:n]
        lps, ids = runner.decode_topk([b[1][-1] for b in beams], [T + len(b[1]) - 1 for b in beams], cur_slots,
                                      kk)
        lps, ids = lps.cpu(), ids.cpu()
        cands = []
        for i, (score, toks) in enumerate(beams):
            for r in range(kk):
                cands.append((score + float(lps[i, r]) - diversity_rate * r, score + float(lps[i, r]), i,
                              int(ids[i, r])))
        cands.sort(key=lambda c: -c[0])
        new_beams, parents = [], []
        for ranked, cum, parent, tok in cands:
            toks = beams[parent][1] + [tok]
            if end_id is not None and tok == end_id:
                finished.append((cum, toks))
            else:
                new_beams.append((cum, toks))
                parents.append(parent)
            if len(new_beams) == W:
                break
        step += 1
        if len(finished) >= W and new_beams:  # early stop when no running beam can beat the finished pool
            best_fin = max(_norm(c, len(t), len_penalty) for c, t in finished)
            best_run = max(_norm(c, max_new_tokens, len_penalty) if len_penalty > 0 else _norm(c, len(t), len_penalty)
                           for c, t in new_beams)
            if best_fin >= best_run:
                beams = []
                break
        # re-order the cache rows: new beam j continues parent's history
        if parents != list(range(len(parents))):
            runner.copy_slots(slots[:len(parents)], [slots[p] for p in parents], T + len(new_beams[0][1]) - 1)
        beams = new_beams
    pool = finished + beams
    pool.sort(key=lambda h: -_norm(h[0], len(h[1]), len_penalty))
    pool = pool[:n_return]
    return BeamResult([t for _, t in pool], [_norm(c, len(t), len_penalty) for c, t in pool], [c for c, _ in pool])


def _norm(cum: float, length: int, len_penalty: float) -> float:
    return cum / (max(length, 1) ** len_penalty)


__all__ = ["beam_search", "BeamResult"]
