"""Continuous-batching LLM engine over ``ModelRunner``.

Replaces what the reference delegates to FasterTransformer-on-Triton
(online-inference/fastertransformer), DeepSpeed-Inference
(bloom-176b-deepspeed) and HF ``pipeline``/``generate`` (inference.py:67-96,
bloom.py:57-77, kserve_api.py:47-72): requests join and leave the running batch
every step (iteration-level scheduling), each request owns one KV-cache slot,
sampling parameters are per request (FT's per-request runtime_top_k / top_p /
temperature / repetition_penalty / random_seed / bad_words / stop_words /
output log-probs).

``step()`` = admit waiting requests (prefill + first token) while slots and
KV pages are free, then one fused decode step for every running request.
One-step lookahead (``pipeline``, on with a pipelining runner): a step launches
the next decode -- its input tokens chained on the device from the step in
flight (``ModelRunner.decode_async``) -- and only then reads the in-flight
step's tokens, so stop checks, streaming callbacks and row preparation overlap
the GPU instead of idling it. A request that stops on a token the host has not
seen yet gets one discarded extra token computed; length stops are predicted
and never over-run.
Chunked prefill (``prefill_chunk``): while requests are decoding, a step
spends at most ``prefill_chunk`` prompt tokens on prefill -- a long prompt is
prefilled over several steps (``ModelRunner.prefill(..., start=)`` continues
its slot), each followed by the decode step of the running batch, so a
2048-token admission no longer stalls every running stream for its whole
prefill; with nothing decoding a prompt prefills in one pass.
Admission reserves a request's worst-case page count (prompt + max_new_tokens)
against the paged cache, so a running request never runs out of pages (no
preemption needed); pages go back to the pool the step a request finishes.
Admitted prompts of different lengths prefill together, right-padded into a
few length-sorted batches (``_prefill_groups``). ``start()`` runs
the loop on a background thread for the HTTP servers; ``generate()`` is the
synchronous batch API used by the finetuner sampler and the evaluator.
"""
from __future__ import annotations

import dataclasses
import itertools
import random
import threading
import time
from concurrent.futures import Future

import torch

from .runner import ModelRunner, mix_seed


@dataclasses.dataclass
class SamplingParams:
    max_new_tokens: int = 50
    min_new_tokens: int = 0
    do_sample: bool = True
    temperature: float = 1.0
    top_k: int = 0
    top_p: float = 1.0
    repetition_penalty: float = 1.0
    seed: int | None = None
    eos_token_id: int | None = None
    stop_sequences: list | None = None   # list of token-id lists (FT stop_words_list)
    bad_words_ids: list | None = None    # list of token-id lists (FT bad_words_list / HF bad_words_ids)
    logprobs: bool = False


@dataclasses.dataclass
class Request:
    rid: int
    prompt: list
    params: SamplingParams
    output: list = dataclasses.field(default_factory=list)
    logprobs: list = dataclasses.field(default_factory=list)
    finish_reason: str | None = None
    slot: int = -1
    seed: int = 0
    t_arrive: float = 0.0
    t_first: float = 0.0
    t_done: float = 0.0
    future: Future | None = None
    on_token: object = None  # callable(request) after every generated token (streaming front ends)
    prefilled: int = 0       # chunked prefill: prompt tokens already in the KV cache

    @property
    def done(self) -> bool:
        return self.finish_reason is not None

    @property
    def tokens(self) -> list:
        return self.prompt + self.output


class LLMEngine:
    def __init__(self, model, max_slots: int = 32, max_len: int | None = None, use_graphs: bool | None = None,
                 max_prefill_tokens: int = 16384, runner=None, page_size: int | None = None,
                 kv_pages: int | None = None, prefill_chunk: int | None = None, pipeline: bool | None = None):
        # ``runner``: e.g. a tp_driver.CollectiveRunner that mirrors every call to TP follower ranks
        self.runner = runner or ModelRunner(model, max_slots=max_slots, max_len=max_len, use_graphs=use_graphs,
                                            page_size=page_size, kv_pages=kv_pages)
        max_slots = self.runner.max_slots
        self.max_len = self.runner.max_len
        self.free = list(range(max_slots))[::-1]
        self.waiting: list[Request] = []
        self.running: list[Request] = []
        self._ids = itertools.count()
        self._lock = threading.Lock()
        self._step_lock = threading.Lock()
        self._wake = threading.Event()
        self._thread = None
        self._stop = False
        self.max_prefill_tokens = max_prefill_tokens
        # prompt-token budget of a step while requests are decoding (None/0: whole prompts)
        self.prefill_chunk = int(prefill_chunk) if prefill_chunk else 0
        self.prefilling: list[Request] = []  # admitted, prompt partially in the cache (r.prefilled tokens)
        self.pipeline = bool(getattr(self.runner, "pipelined", False)) if pipeline is None else pipeline
        self._inflight = None  # (DecodeHandle, [Request]) of the launched, not yet read decode step
        self.stats = {"steps": 0, "decode_tokens": 0, "prefill_tokens": 0, "finished": 0, "prefill_batches": 0,
                      "prefill_pad_tokens": 0, "prefill_chunks": 0, "max_step_prefill_tokens": 0,
                      "decode_steps": 0}
        cache = getattr(self.runner, "cache", None)
        self._paged = cache is not None and getattr(cache, "paged", False)
        self._page_budget = cache.n_pages if self._paged else 0
        self._committed = 0  # worst-case pages promised to admitted requests

    # ------------------------------------------------------------ requests
    def add_request(self, prompt: list, params: SamplingParams, future: Future | None = None,
                    on_token=None) -> Request:
        prompt = [int(t) for t in prompt]
        if not prompt:
            raise ValueError("empty prompt")
        if len(prompt) >= self.max_len:
            prompt = prompt[-(self.max_len - 1):]
        seed = params.seed if params.seed is not None else random.getrandbits(63)
        r = Request(next(self._ids), prompt, params, seed=seed, t_arrive=time.perf_counter(), future=future,
                    on_token=on_token)
        if params.max_new_tokens <= 0:
            r.finish_reason = "length"
            r.t_done = r.t_arrive
            if future is not None:
                future.set_result(r)
            return r
        with self._lock:
            self.waiting.append(r)
        self._wake.set()
        return r

    def has_work(self) -> bool:
        return bool(self.waiting or self.running or self.prefilling or self._inflight)

    def _row(self, r: Request, token: int | None = None, ahead: int = 0) -> dict:
        """Decode-row parameters. ``ahead`` = 1: the row's input token is the
        in-flight step's (not yet on the host), chained on the device."""
        p = r.params
        n_gen = len(r.output) + ahead
        greedy = (not p.do_sample) or p.temperature <= 0
        bans = []
        for w in p.bad_words_ids or ():
            if len(w) == 1:
                bans.append(int(w[0]))
            elif len(w) > 1 and r.tokens[-(len(w) - 1):] == list(w[:-1]):
                bans.append(int(w[-1]))
        if p.eos_token_id is not None and n_gen < p.min_new_tokens:
            bans.append(int(p.eos_token_id))
        if ahead:
            return {"token": None, "pos": len(r.tokens) - 1 + ahead,
                    "slot": r.slot, "temperature": 0.0 if greedy else float(p.temperature),
                    "top_k": int(p.top_k or 0), "top_p": float(p.top_p if p.top_p is not None else 1.0),
                    "rep": float(p.repetition_penalty or 1.0), "seed": mix_seed(r.seed, n_gen), "bans": bans}
        return {"token": token if token is not None else r.tokens[-1], "pos": len(r.tokens) - 1,
                "slot": r.slot, "temperature": 0.0 if greedy else float(p.temperature),
                "top_k": int(p.top_k or 0), "top_p": float(p.top_p if p.top_p is not None else 1.0),
                "rep": float(p.repetition_penalty or 1.0), "seed": mix_seed(r.seed, n_gen), "bans": bans}

    def _append(self, r: Request, tok: int, lp: float):
        r.output.append(int(tok))
        if r.params.logprobs:
            r.logprobs.append(float(lp))
        p = r.params
        if len(r.output) == 1:
            r.t_first = time.perf_counter()
        if p.eos_token_id is not None and tok == p.eos_token_id and len(r.output) > p.min_new_tokens:
            r.finish_reason = "stop"
        elif any(s and r.output[-len(s):] == list(s) for s in (p.stop_sequences or ())):
            r.finish_reason = "stop"
        elif len(r.output) >= p.max_new_tokens or len(r.tokens) >= self.max_len:
            r.finish_reason = "length"
        if r.on_token is not None:
            try:
                r.on_token(r)
            except Exception:  # noqa: BLE001 -- a broken stream consumer must not stall the batch
                r.on_token = None

    def _pages_needed(self, r: Request) -> int:
        if not self._paged:
            return 0
        return self.runner.cache.pages_for(min(len(r.prompt) + r.params.max_new_tokens, self.max_len))

    def _free_slot(self, r: Request):
        if r.slot >= 0:
            self.runner.release(r.slot)
            self.free.append(r.slot)
            r.slot = -1
            self._committed -= self._pages_needed(r)

    def _finish(self, r: Request):
        r.t_done = time.perf_counter()
        self._free_slot(r)
        self.stats["finished"] += 1
        if r.future is not None and not r.future.done():
            r.future.set_result(r)

    # ---------------------------------------------------------------- step
    def beam_generate(self, prompt: list, num_beams: int, max_new_tokens: int, eos_token_id: int | None = None,
                      len_penalty: float = 1.0, diversity_rate: float = 0.0, n_return: int = 1):
        """Beam search for one prompt on ``num_beams`` slots of this engine's cache
        (mutually exclusive with ``step``; FT beam_width > 1 requests)."""
        from .beam import beam_search
        # a tensor-parallel runner (tp_driver.CollectiveRunner) mirrors prefill / decode_topk /
        # copy_slots / release to its followers, so beams run under TP unchanged
        need = 0
        if self._paged:
            need = num_beams * (self.runner.cache.pages_for(min(len(prompt) + max_new_tokens, self.max_len)) + 1)
        with self._step_lock:
            self._drain([])  # the in-flight lookahead step finishes before the beams take the runner
            with self._lock:
                if len(self.free) < num_beams:
                    raise RuntimeError(f"need {num_beams} free cache slots, have {len(self.free)}")
                if self._committed + need > self._page_budget and self._paged:
                    raise RuntimeError(f"need {need} free KV pages, have {self._page_budget - self._committed}")
                slots = [self.free.pop() for _ in range(num_beams)]
                self._committed += need
            try:
                return beam_search(self.runner, [int(t) for t in prompt], slots, max_new_tokens, eos_token_id,
                                   len_penalty, diversity_rate, n_return)
            finally:
                with self._lock:
                    for s_ in slots:
                        self.runner.release(s_)
                    self.free.extend(slots)
                    self._committed -= need

    def step(self) -> list[Request]:
        """Admit + one decode step. Returns the requests that finished."""
        with self._step_lock:
            return self._step()

    def _first_token(self, r: Request, logits, finished: list):
        toks, lps = self.runner.sample_first(logits, [self._row(r, 0)])
        self._append(r, toks[0], lps[0])
        if r.done:
            self._finish(r)
            finished.append(r)
        else:
            self.running.append(r)

    def _chunk_step(self, budget: int, finished: list) -> int:
        """Advance partially prefilled prompts by up to ``budget`` tokens."""
        used = 0
        for r in list(self.prefilling):
            if used >= budget:
                break
            p0 = r.prefilled
            n = min(budget - used, len(r.prompt) - p0)
            ids = torch.tensor([r.prompt[p0:p0 + n]], dtype=torch.long)
            logits = self.runner.prefill(ids, [r.slot], [n], start=[p0])
            r.prefilled += n
            used += n
            self.stats["prefill_tokens"] += n
            self.stats["prefill_chunks"] += 1
            if r.prefilled == len(r.prompt):
                self.prefilling.remove(r)
                self._first_token(r, logits, finished)
        return used

    def _step(self) -> list[Request]:
        finished = []
        chunked = self.prefill_chunk > 0 and (self.running or self.prefilling)
        budget = self.prefill_chunk if chunked else self.max_prefill_tokens
        used = self._chunk_step(budget, finished) if self.prefilling else 0
        budget -= used
        with self._lock:
            admit = []
            while self.waiting and self.free and budget > 0 and (not admit or budget >= len(self.waiting[0].prompt)):
                need = self._pages_needed(self.waiting[0])
                if self._paged and self._committed + need > self._page_budget:
                    if need > self._page_budget:  # can never fit: fail it rather than block the queue
                        r = self.waiting.pop(0)
                        r.finish_reason = "error"
                        r.t_done = time.perf_counter()
                        if r.future is not None and not r.future.done():
                            r.future.set_exception(RuntimeError(
                                f"request needs {need} KV pages > cache size {self._page_budget}"))
                        continue
                    break
                r = self.waiting.pop(0)
                r.slot = self.free.pop()
                self._committed += need
                if chunked and len(r.prompt) > budget:  # prefill this one chunk by chunk
                    r.prefilled = 0
                    self.prefilling.append(r)
                    break
                budget -= len(r.prompt)
                admit.append(r)
        if self.prefilling and budget > 0 and chunked:
            used += self._chunk_step(budget, finished)
        for group in _prefill_groups(admit):
            T = max(len(r.prompt) for r in group)
            lens = [len(r.prompt) for r in group]
            ids = torch.tensor([r.prompt + [0] * (T - len(r.prompt)) for r in group], dtype=torch.long)
            if all(L == T for L in lens):
                logits = self.runner.prefill(ids, [r.slot for r in group])
            else:
                logits = self.runner.prefill(ids, [r.slot for r in group], lens)
            toks, lps = self.runner.sample_first(logits, [self._row(r, 0) for r in group])
            self.stats["prefill_tokens"] += sum(lens)
            used += sum(lens)
            self.stats["prefill_pad_tokens"] += T * len(group) - sum(lens)
            self.stats["prefill_batches"] += 1
            for r, t, lp in zip(group, toks, lps):
                self._append(r, t, lp)
                if r.done:
                    self._finish(r)
                    finished.append(r)
                else:
                    self.running.append(r)
        # decode one token for everything already running (incl. just admitted)
        if self.pipeline and self._lookahead_ok():
            self._decode_lookahead(finished)
        elif self.running or self._inflight:
            self._drain(finished)
            # the drained step may have finished requests (slot released, pages freed)
            self.running = [r for r in self.running if not r.done]
            rows = [self._row(r) for r in self.running]
            if rows:
                toks, lps = self.runner.decode(rows)
                self.stats["decode_tokens"] += len(rows)
                self.stats["decode_steps"] += 1
                self._take(self.running, toks, lps, finished)
            self.running = [r for r in self.running if not r.done]
        self.stats["steps"] += 1
        self.stats["max_step_prefill_tokens"] = max(self.stats["max_step_prefill_tokens"], used)
        return finished

    # ------------------------------------------------------------ lookahead
    def _take(self, reqs, toks, lps, finished):
        for r, t, lp in zip(reqs, toks, lps):
            if r.done:  # stopped on the previous token: this one was computed ahead and is dropped
                continue
            self._append(r, t, lp)
            if r.done:
                self._finish(r)
                finished.append(r)

    def _drain(self, finished):
        """Read the in-flight decode step (before a synchronous runner call)."""
        if self._inflight is not None:
            h, reqs = self._inflight
            self._inflight = None
            toks, lps = h.result()
            self._take(reqs, toks, lps, finished)

    def _lookahead_ok(self) -> bool:
        # a multi-token bad word's ban depends on the token still in flight
        return not any(len(w) > 1 for r in self.running for w in (r.params.bad_words_ids or ()))

    def _last_by_length(self, r: Request, ahead: int) -> bool:
        return (len(r.output) + ahead >= r.params.max_new_tokens
                or len(r.tokens) + ahead >= self.max_len)

    def _decode_lookahead(self, finished):
        """Launch step t+1 (tokens of step t chained on the device), then read step t."""
        inflight = self._inflight
        src = {id(r): i for i, r in enumerate(inflight[1])} if inflight else {}
        rows, reqs = [], []
        for r in self.running:
            if r.done:
                continue
            j = src.get(id(r))
            if j is None:
                rows.append(self._row(r))
            else:
                if self._last_by_length(r, 1):  # its in-flight token is its last one
                    continue
                row = self._row(r, ahead=1)
                row["src"] = j
                rows.append(row)
            reqs.append(r)
        h = self.runner.decode_async(rows, prev=inflight[0] if inflight else None) if rows else None
        if rows:
            self.stats["decode_tokens"] += len(rows)
            self.stats["decode_steps"] += 1
        self._inflight = None
        if inflight is not None:
            toks, lps = inflight[0].result()
            self._take(inflight[1], toks, lps, finished)
        self._inflight = (h, reqs) if h is not None else None
        self.running = [r for r in self.running if not r.done]

    def run_until_done(self, reqs: list[Request] | None = None):
        while self.has_work() and (reqs is None or not all(r.done for r in reqs)):
            self.step()

    def generate(self, prompts: list[list[int]], params: SamplingParams | list[SamplingParams]) -> list[Request]:
        ps = params if isinstance(params, list) else [params] * len(prompts)
        reqs = [self.add_request(p, sp) for p, sp in zip(prompts, ps)]
        self.run_until_done(reqs)
        return reqs

    # ------------------------------------------------------ background loop
    def submit(self, prompt: list, params: SamplingParams, on_token=None) -> Future:
        if self._thread is None:
            self.start()
        fut: Future = Future()
        self.add_request(prompt, params, fut, on_token=on_token)
        return fut

    def start(self):
        if self._thread is not None:
            return
        self._stop = False
        self._thread = threading.Thread(target=self._loop, name="llm-engine", daemon=True)
        self._thread.start()

    def stop(self):
        self._stop = True
        self._wake.set()
        if self._thread is not None:
            self._thread.join()
            self._thread = None

    def _loop(self):
        dev = self.runner.device
        if dev.type == "cuda":
            torch.cuda.set_device(dev)
        while not self._stop:
            if not self.has_work():
                self._wake.wait(0.05)
                self._wake.clear()
                continue
            try:
                self.step()
            except Exception as e:  # fail every in-flight request, keep serving
                with self._lock:
                    victims = self.running + self.prefilling + self.waiting
                    self.running, self.prefilling, self.waiting = [], [], []
                    self._inflight = None
                for r in victims:
                    try:
                        self._free_slot(r)
                    except Exception:  # noqa: BLE001 -- a broken runner must not stop the loop
                        r.slot = -1
                    if r.future is not None and not r.future.done():
                        r.future.set_exception(e)


def _prefill_groups(reqs: list[Request], slack: float = 0.25, min_slack: int = 256) -> list[list[Request]]:
    """Length-sorted batches whose right padding stays within ``slack`` of the
    real tokens (or ``min_slack`` tokens: short prompts are launch-bound, so
    they batch freely)."""
    out, cur, real = [], [], 0
    for r in sorted(reqs, key=lambda r: len(r.prompt)):
        L = len(r.prompt)
        if cur and L * (len(cur) + 1) - (real + L) > max(slack * (real + L), min_slack):
            out.append(cur)
            cur, real = [], 0
        cur.append(r)
        real += L
    if cur:
        out.append(cur)
    return out


__all__ = ["LLMEngine", "SamplingParams", "Request"]
