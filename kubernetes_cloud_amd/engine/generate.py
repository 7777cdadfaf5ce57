"""Batch generation API on the continuous-batching engine.

Serves the finetuner's periodic sampler (finetuner.py:538-630, 835-881) and
the evaluator CLI (evaluator.py:175-219) -- HF ``generate`` semantics
(num_return_sequences, bad_words_ids, min length, repetition penalty, top-k/p)
over ``LLMEngine`` with a KV cache sized for this call.
"""
from __future__ import annotations

import dataclasses

import torch

from .llm_engine import LLMEngine, SamplingParams


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

    def sampling_params(self, seed: int | None = None) -> SamplingParams:
        return SamplingParams(max_new_tokens=self.max_new_tokens, min_new_tokens=self.min_new_tokens,
                              do_sample=self.do_sample, temperature=self.temperature, top_k=self.top_k,
                              top_p=self.top_p, repetition_penalty=self.repetition_penalty, seed=seed,
                              eos_token_id=self.eos_token_id, stop_sequences=self.stop_sequences,
                              bad_words_ids=self.bad_words_ids, logprobs=self.return_logprobs)


@dataclasses.dataclass
class GenerationResult:
    sequences: torch.Tensor        # [N, prompt + new] (padded with pad id after stop)
    lengths: torch.Tensor          # [N] total valid length
    logprobs: torch.Tensor | None  # [N, new]
    prompt_len: int


@torch.no_grad()
def generate(model, input_ids: torch.Tensor, cfg: GenerationConfig, use_graphs: bool = False) -> GenerationResult:
    """``input_ids``: [B, T] prompts (one request's samples); sequences come back
    in input order, ``num_return_sequences`` consecutive rows per prompt."""
    ids = input_ids.tolist()
    prompts = [p for p in ids for _ in range(cfg.num_return_sequences)]
    N, T = len(prompts), input_ids.shape[1]
    eng = LLMEngine(model, max_slots=N, max_len=min(T + cfg.max_new_tokens, max(model.cfg.max_pos, T + 1)),
                    use_graphs=use_graphs)
    params = [cfg.sampling_params(None if cfg.seed is None else cfg.seed + i) for i in range(N)]
    reqs = eng.generate(prompts, params)
    pad = cfg.pad_token_id if cfg.pad_token_id is not None else (cfg.eos_token_id or 0)
    width = T + max(len(r.output) for r in reqs)
    seqs = torch.full((N, width), pad, dtype=torch.long)
    lps = torch.zeros(N, width - T) if cfg.return_logprobs else None
    lens = torch.empty(N, dtype=torch.long)
    for i, r in enumerate(reqs):
        toks = r.prompt + r.output
        seqs[i, :len(toks)] = torch.tensor(toks)
        lens[i] = len(toks)
        if lps is not None and r.logprobs:
            lps[i, :len(r.logprobs)] = torch.tensor(r.logprobs)
    return GenerationResult(seqs, lens, lps, T)


__all__ = ["GenerationConfig", "GenerationResult", "generate"]
