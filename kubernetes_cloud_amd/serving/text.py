"""Text-generation front end: model loading + an HF-``pipeline``-compatible
generator over the continuous-batching engine.

Every LLM predictor of the reference funnels into ``transformers.pipeline(
"text-generation")`` or ``model.generate`` (finetuner/inference.py:67-96,
bloom-176b/model/bloom.py:57-77, tensorizer-isvc kserve_api.py:47-72 and
flask_api.py:31-45, custom-pytorch-aitextgen model.py:16-21). ``TextGenerator``
accepts the same keyword arguments (HF semantics: ``max_length`` and
``min_length`` count the prompt, ``top_k`` defaults to 50, ``do_sample``
defaults to False, ``stop_sequence``) and returns the same
``[{"generated_text": ...}]`` structure, but every request is a row of the
shared engine batch instead of a separate ``generate`` call.
"""
from __future__ import annotations

import logging
import os
import time

import torch

from ..engine.llm_engine import LLMEngine, SamplingParams

log = logging.getLogger("kca.serving")


def load_lm(path: str, device=None, dtype=torch.bfloat16, tensors_file: str | None = None,
            random_init: bool = False):
    """-> (model, tokenizer). ``path``: HF-layout directory (config.json +
    safetensors/bin + tokenizer) or a preset name with ``random_init``.
    ``tensors_file``: stream weights from our ``.tensors`` file -- or an
    ``http(s)://`` / ``s3://`` URI -- straight into HBM (the tensorizer path,
    load_model.py:46-73) instead of safetensors."""
    from ..io.hf import load_pretrained, load_tokenizer
    from ..models.causal_lm import build_model
    from ..models.config import PRESETS_HF, preset
    dev = torch.device(device) if device is not None else (
        torch.device("cuda", 0) if torch.cuda.is_available() else torch.device("cpu"))
    if dev.type == "cpu" and dtype in (torch.bfloat16, torch.float16):
        dtype = torch.float32
    t0 = time.perf_counter()
    tok = None
    if tensors_file and not os.path.isdir(path):
        # URI-only load (s3:// / https:// / a file): config from the file's metadata
        from ..io.hf import load_tensorized
        model, stats = load_tensorized(tensors_file, None, device=dev, dtype=dtype)
        log.info("tensorized load: %s", stats)
    elif os.path.isdir(path):
        if tensors_file:
            from ..io.hf import load_tensorized
            model, stats = load_tensorized(tensors_file, path, device=dev, dtype=dtype)
            log.info("tensorized load: %s", stats)
        else:
            model = load_pretrained(path, device=dev, dtype=dtype, random_init_if_missing=random_init)
        try:
            tok = load_tokenizer(path)
        except Exception as e:  # noqa: BLE001
            log.warning("no tokenizer in %s (%s)", path, e)
    elif random_init and (path in PRESETS_HF or path.split("/")[-1].lower() in PRESETS_HF):
        name = path if path in PRESETS_HF else path.split("/")[-1].lower()
        model = build_model(preset(name), device=dev, dtype=dtype, seed=0)
    else:
        raise FileNotFoundError(f"{path}: not a model directory (no network: HF hub IDs cannot be fetched)")
    log.info("loaded %s in %.2fs", path, time.perf_counter() - t0)
    return model.eval(), tok


class TextGenerator:
    def __init__(self, model, tokenizer, max_slots: int = 32, use_graphs: bool | None = None,
                 background: bool = True, max_len: int | None = None, runner=None):
        self.model, self.tokenizer = model, tokenizer
        self.engine = LLMEngine(model, max_slots=max_slots, max_len=max_len or model.cfg.max_pos,
                                use_graphs=use_graphs, runner=runner)
        self.background = background
        if background:
            self.engine.start()

    def close(self):
        self.engine.stop()

    # ------------------------------------------------------------ params
    def sampling_params(self, prompt_len: int, *, max_new_tokens=None, max_length=None, min_length=None,
                        min_new_tokens=None, do_sample=None, temperature=None, top_k=None, top_p=None,
                        repetition_penalty=None, seed=None, eos_token_id=None, stop_sequence=None,
                        bad_words=None, bad_words_ids=None, logprobs=False, **ignored) -> SamplingParams:
        for k, v in ignored.items():
            if v is not None and k not in ("typical_p", "penalty_alpha", "num_return_sequences", "pad_token_id"):
                log.debug("ignoring unsupported generation kwarg %s=%r", k, v)
        tok = self.tokenizer
        if max_new_tokens is None:
            max_new_tokens = (max_length - prompt_len) if max_length is not None else 20
        if min_new_tokens is None:
            min_new_tokens = max(0, (min_length or 0) - prompt_len)
        eos = eos_token_id if eos_token_id is not None else (tok.eos_token_id if tok is not None else None)
        stops = None
        if stop_sequence:
            ids = tok.encode(stop_sequence, add_special_tokens=False)
            stops = [ids] if ids else None
        bw = [list(w) for w in (bad_words_ids or [])]
        for w in bad_words or []:
            if isinstance(w, str):
                ids = tok.encode(w, add_special_tokens=False)
                if ids:
                    bw.append(ids)
            elif isinstance(w, (list, tuple)):
                bw.append([int(t) for t in w])
        return SamplingParams(
            max_new_tokens=max(0, int(max_new_tokens)), min_new_tokens=int(min_new_tokens),
            do_sample=bool(do_sample) if do_sample is not None else False,
            temperature=1.0 if temperature is None else float(temperature),
            top_k=50 if top_k is None else int(top_k), top_p=1.0 if top_p is None else float(top_p),
            repetition_penalty=1.0 if repetition_penalty is None else float(repetition_penalty),
            seed=seed, eos_token_id=eos, stop_sequences=stops, bad_words_ids=bw or None, logprobs=logprobs)

    # -------------------------------------------------------------- run
    def generate_ids(self, prompts: list[list[int]], params: list[SamplingParams], on_token=None):
        """``on_token(index, request)`` is called from the engine thread after
        every generated token of request ``index`` (streaming responses)."""
        cbs = [None] * len(prompts) if on_token is None else \
            [(lambda r, i=i: on_token(i, r)) for i in range(len(prompts))]
        if self.background:
            futs = [self.engine.submit(p, sp, on_token=cb) for p, sp, cb in zip(prompts, params, cbs)]
            return [f.result() for f in futs]
        reqs = [self.engine.add_request(p, sp, on_token=cb) for p, sp, cb in zip(prompts, params, cbs)]
        self.engine.run_until_done(reqs)
        return reqs

    async def agenerate_ids(self, prompts: list[list[int]], params: list[SamplingParams]):
        """``generate_ids`` for an event loop: the requests go to the background engine and the
        caller awaits their futures (no thread blocked while they generate)."""
        import asyncio
        if not self.background:
            return await asyncio.get_running_loop().run_in_executor(None, self.generate_ids, prompts, params)
        futs = [self.engine.submit(p, sp) for p, sp in zip(prompts, params)]
        return list(await asyncio.gather(*(asyncio.wrap_future(f) for f in futs)))

    def _prepare(self, text_inputs, num_return_sequences: int = 1, **kw):
        single = isinstance(text_inputs, str)
        texts = [text_inputs] if single else list(text_inputs)
        tok = self.tokenizer
        enc = [tok.encode(t) for t in texts]
        prompts, params = [], []
        seed = kw.pop("seed", None)
        for i, ids in enumerate(enc):
            for j in range(num_return_sequences or 1):
                prompts.append(ids)
                s = None if seed is None else int(seed) + i * 1000 + j
                params.append(self.sampling_params(len(ids), seed=s, **kw))
        return single, texts, enc, prompts, params

    def _finish(self, reqs, single, texts, enc, return_full_text: bool, num_return_sequences: int):
        tok = self.tokenizer
        out, k = [], 0
        for t, ids in zip(texts, enc):
            group = []
            for _ in range(num_return_sequences or 1):
                r = reqs[k]
                k += 1
                full = tok.decode(r.prompt + r.output, skip_special_tokens=True)
                plen = len(tok.decode(r.prompt, skip_special_tokens=True))
                new = full[plen:]
                group.append({"generated_text": (t + new) if return_full_text else new})
            out.append(group)
        return out[0] if single else out

    def __call__(self, text_inputs, return_full_text: bool = True, num_return_sequences: int = 1, **kw):
        single, texts, enc, prompts, params = self._prepare(text_inputs, num_return_sequences, **kw)
        return self._finish(self.generate_ids(prompts, params), single, texts, enc, return_full_text,
                            num_return_sequences)

    async def acall(self, text_inputs, return_full_text: bool = True, num_return_sequences: int = 1, **kw):
        single, texts, enc, prompts, params = self._prepare(text_inputs, num_return_sequences, **kw)
        return self._finish(await self.agenerate_ids(prompts, params), single, texts, enc, return_full_text,
                            num_return_sequences)


__all__ = ["load_lm", "TextGenerator"]
