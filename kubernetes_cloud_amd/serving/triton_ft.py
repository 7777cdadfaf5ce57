"""FasterTransformer-compatible Triton endpoint + model-store tooling (S6/S7).

The reference serves GPT-J-6B / GPT-NeoX-20B with Triton's FasterTransformer
backend (online-inference/fastertransformer): a model store
``triton-model-store/fastertransformer/{config.pbtxt, 1/}`` built by the
download job (download-weights-job-gptj.yml:30-250) and V2 requests with FT's
tensor names (client/example.py:63-152, client/sample_request.json).

``FasterTransformerModel`` is a V2 ``Model`` named ``fastertransformer`` that
accepts exactly those tensors -- input_ids, input_lengths, request_output_len,
start_id, end_id, runtime_top_k, runtime_top_p, temperature, len_penalty,
repetition_penalty, random_seed, is_return_log_probs, beam_width,
beam_search_diversity_rate, bad_words_list, stop_words_list,
prompt_learning_task_name_ids -- and returns output_ids [B, beam, L],
sequence_length [B, beam], cum_log_probs [B, beam], output_log_probs
[B, beam, out_len]; each batch row becomes one request of the engine's
continuous batch. FT conventions kept: ``runtime_top_k == 0 and runtime_top_p
== 0`` is greedy, ``runtime_top_p == 0`` disables nucleus, word lists are
``[B, 2, L]`` (flattened ids + cumulative end offsets, -1 padded), output_ids
holds prompt + generation padded with end_id.

``write_model_store`` is the converter half of the download job: an HF
checkpoint directory becomes a store whose ``1/`` holds our ``model.tensors``
(streamed into HBM at load) + config + tokenizer, and whose config.pbtxt
carries FT's schema and parameters (tensor_para_size, data_type, model_type,
model_checkpoint_path).
"""
from __future__ import annotations

import json
import logging
import os
import re

import numpy as np

from .server import InvalidInput, Model

log = logging.getLogger("kca.serving")

FT_INPUTS = [
    ("input_ids", "TYPE_INT32", "[ -1 ]", False), ("start_id", "TYPE_INT32", "[ 1 ]", True),
    ("end_id", "TYPE_INT32", "[ 1 ]", True), ("input_lengths", "TYPE_INT32", "[ 1 ]", False),
    ("request_output_len", "TYPE_INT32", "[ -1 ]", False), ("runtime_top_k", "TYPE_INT32", "[ 1 ]", True),
    ("runtime_top_p", "TYPE_FP32", "[ 1 ]", True), ("beam_search_diversity_rate", "TYPE_FP32", "[ 1 ]", True),
    ("temperature", "TYPE_FP32", "[ 1 ]", True), ("len_penalty", "TYPE_FP32", "[ 1 ]", True),
    ("repetition_penalty", "TYPE_FP32", "[ 1 ]", True), ("random_seed", "TYPE_UINT64", "[ 1 ]", True),
    ("is_return_log_probs", "TYPE_BOOL", "[ 1 ]", True), ("beam_width", "TYPE_INT32", "[ 1 ]", True),
    ("bad_words_list", "TYPE_INT32", "[ 2, -1 ]", True), ("stop_words_list", "TYPE_INT32", "[ 2, -1 ]", True),
    ("prompt_learning_task_name_ids", "TYPE_UINT32", "[ 1 ]", True),
]
FT_OUTPUTS = [("output_ids", "TYPE_INT32", "[ -1, -1 ]"), ("sequence_length", "TYPE_INT32", "[ -1 ]"),
              ("cum_log_probs", "TYPE_FP32", "[ -1 ]"), ("output_log_probs", "TYPE_FP32", "[ -1, -1 ]")]


# ------------------------------------------------------------- pbtxt
def render_config_pbtxt(params: dict, name: str = "fastertransformer", max_batch_size: int = 1024,
                        default_model_filename: str = "model") -> str:
    lines = [f'name: "{name}"', 'backend: "fastertransformer"', f'default_model_filename: "{default_model_filename}"',
             f"max_batch_size: {max_batch_size}", "", "model_transaction_policy {", "  decoupled: False", "}", "",
             "input ["]
    ins = []
    for n, dt, dims, opt in FT_INPUTS:
        s = f'  {{\n    name: "{n}"\n    data_type: {dt}\n    dims: {dims}\n'
        if dims == "[ 1 ]":
            s += "    reshape: { shape: [ ] }\n"
        if opt:
            s += "    optional: true\n"
        ins.append(s + "  }")
    lines.append(",\n".join(ins))
    lines += ["]", "output ["]
    lines.append(",\n".join(f'  {{\n    name: "{n}"\n    data_type: {dt}\n    dims: {dims}\n  }}'
                            for n, dt, dims in FT_OUTPUTS))
    lines += ["]", "instance_group [", "  {", "    count: 1", "    kind: KIND_CPU", "  }", "]"]
    for k, v in params.items():
        lines.append(f'parameters {{\n  key: "{k}"\n  value: {{\n    string_value: "{v}"\n  }}\n}}')
    return "\n".join(lines) + "\n"


def parse_config_pbtxt(text: str) -> dict:
    """Minimal reader: top-level scalars + ``parameters {key value.string_value}``."""
    out = {"parameters": {}}
    for m in re.finditer(r'parameters\s*\{\s*key:\s*"([^"]+)"\s*value:\s*\{\s*string_value:\s*"([^"]*)"\s*\}\s*\}',
                         text):
        out["parameters"][m.group(1)] = m.group(2)
    for key in ("name", "backend", "default_model_filename"):
        m = re.search(rf'^\s*{key}:\s*"([^"]*)"', text, re.M)
        if m:
            out[key] = m.group(1)
    m = re.search(r"^\s*max_batch_size:\s*(\d+)", text, re.M)
    if m:
        out["max_batch_size"] = int(m.group(1))
    return out


def write_model_store(model_dir: str, store_dir: str, tensor_para_size: int = 1, data_type: str = "fp16",
                      name: str = "fastertransformer") -> str:
    """HF checkpoint dir -> ``{store}/{name}/config.pbtxt`` + ``1/model.tensors``."""
    import torch

    from ..io.hf import load_pretrained
    from ..io.tensors import serialize
    from ..models.config import LMConfig
    cfg = LMConfig.from_pretrained(model_dir)
    dt = {"bf16": torch.bfloat16, "fp16": torch.float16, "fp32": torch.float32}[data_type]
    model = load_pretrained(model_dir, device="cpu", dtype=dt)
    vdir = os.path.join(store_dir, name, "1")
    os.makedirs(vdir, exist_ok=True)
    serialize(model, os.path.join(vdir, "model.tensors"))
    for f in os.listdir(model_dir):
        if f.endswith(".json") and not f.endswith("index.json") or f in ("merges.txt", "vocab.json",
                                                                          "tokenizer.model"):
            with open(os.path.join(model_dir, f), "rb") as a, open(os.path.join(vdir, f), "wb") as b:
                b.write(a.read())
    mtype = {"gptj": "GPT-J", "gpt_neox": "GPT-NeoX", "gpt2": "GPT", "bloom": "BLOOM", "gpt_neo": "GPT-Neo"}.get(
        cfg.arch, cfg.arch)
    params = {"tensor_para_size": str(tensor_para_size), "pipeline_para_size": "1", "data_type": data_type,
              "model_type": mtype, "model_checkpoint_path": os.path.abspath(vdir), "enable_custom_all_reduce": "1"}
    with open(os.path.join(store_dir, name, "config.pbtxt"), "w") as f:
        f.write(render_config_pbtxt(params, name=name))
    return os.path.join(store_dir, name)


# --------------------------------------------------------------- model
def _col(inputs: dict, name: str, B: int, default, dtype=None):
    a = inputs.get(name)
    if a is None:
        return [default] * B
    a = np.asarray(a)
    a = a.reshape(1) if a.ndim == 0 else a.reshape(a.shape[0], -1)[:, 0]
    if len(a) == 1 and B > 1:
        a = np.repeat(a, B)
    if len(a) != B:
        raise InvalidInput(f"{name}: batch {len(a)} != {B}")
    return [dtype(x) if dtype else x for x in a]


def parse_word_list(arr) -> list[list[list[int]]]:
    """FT ``[B, 2, L]`` word lists -> per row list of token-id lists."""
    if arr is None:
        return []
    a = np.asarray(arr)
    if a.ndim == 2:
        a = a[None]
    out = []
    for row in a:
        ids, offs = row[0].tolist(), [int(o) for o in row[1].tolist() if int(o) >= 0]
        words, prev = [], 0
        for end in offs:
            w = [int(t) for t in ids[prev:end]]
            if w:
                words.append(w)
            prev = end
        out.append(words)
    return out


class FasterTransformerModel(Model):
    def __init__(self, name: str = "fastertransformer", generator=None, end_id: int | None = None,
                 store_dir: str | None = None):
        super().__init__(name)
        self.generator, self.store_dir = generator, store_dir
        self.end_id = end_id
        self.config: dict = {}
        if generator is not None:
            self.ready = True
            if self.end_id is None and generator.tokenizer is not None:
                self.end_id = generator.tokenizer.eos_token_id

    def load(self):
        from .text import TextGenerator, load_lm
        path = os.path.join(self.store_dir, self.name, "config.pbtxt")
        with open(path) as f:
            self.config = parse_config_pbtxt(f.read())
        ck = self.config["parameters"].get("model_checkpoint_path") or os.path.join(self.store_dir, self.name, "1")
        tp = int(self.config["parameters"].get("tensor_para_size", "1"))
        if tp != 1:
            log.warning("tensor_para_size=%d: serve with the TP launcher (serving.tp_server); loading TP=1", tp)
        # the store's data_type is the serving precision (FT's default fp16): the decode step runs it natively
        # (fp16 instantiations of every decode kernel), no conversion to bf16 at load
        import torch
        dt = {"fp16": torch.float16, "bf16": torch.bfloat16, "fp32": torch.float32}[
            self.config["parameters"].get("data_type", "fp16")]
        model, tok = load_lm(ck, dtype=dt, tensors_file=os.path.join(ck, "model.tensors"))
        self.generator = TextGenerator(model, tok, max_slots=int(os.getenv("MAX_BATCH", 64)))
        if self.end_id is None:
            self.end_id = tok.eos_token_id if tok is not None else model.cfg.vocab_size - 1
        self.ready = True

    def metadata(self) -> dict:
        m = {"TYPE_INT32": "INT32", "TYPE_FP32": "FP32", "TYPE_UINT64": "UINT64", "TYPE_BOOL": "BOOL",
             "TYPE_UINT32": "UINT32"}
        return {"name": self.name, "versions": ["1"], "platform": "fastertransformer",
                "inputs": [{"name": n, "datatype": m[d], "shape": [-1] + json.loads(s.replace(" ", ""))}
                           for n, d, s, _ in FT_INPUTS],
                "outputs": [{"name": n, "datatype": m[d], "shape": [-1] + json.loads(s.replace(" ", ""))}
                            for n, d, s in FT_OUTPUTS]}

    def _prepare(self, inputs: dict):
        from ..engine.llm_engine import SamplingParams
        if "input_ids" not in inputs or "request_output_len" not in inputs:
            raise InvalidInput("input_ids and request_output_len are required")
        ids = np.asarray(inputs["input_ids"]).astype(np.int64)
        if ids.ndim == 1:
            ids = ids[None]
        B = ids.shape[0]
        lens = _col(inputs, "input_lengths", B, ids.shape[1], int)
        out_len = _col(inputs, "request_output_len", B, 16, int)
        end_id = _col(inputs, "end_id", B, self.end_id, int)
        top_k = _col(inputs, "runtime_top_k", B, 1, int)
        top_p = _col(inputs, "runtime_top_p", B, 0.0, float)
        temp = _col(inputs, "temperature", B, 1.0, float)
        rep = _col(inputs, "repetition_penalty", B, 1.0, float)
        seed = _col(inputs, "random_seed", B, 0, int)
        beam = _col(inputs, "beam_width", B, 1, int)
        want_lp = any(bool(x) for x in _col(inputs, "is_return_log_probs", B, False, bool))
        bad = parse_word_list(inputs.get("bad_words_list"))
        stop = parse_word_list(inputs.get("stop_words_list"))
        if bad and len(bad) == 1 and B > 1:
            bad = bad * B
        if stop and len(stop) == 1 and B > 1:
            stop = stop * B
        lpen = _col(inputs, "len_penalty", B, 1.0, float)
        div = _col(inputs, "beam_search_diversity_rate", B, 0.0, float)
        prompts, params = [], []
        for b in range(B):
            p = ids[b, :lens[b]].tolist()
            greedy = top_k[b] == 0 and top_p[b] == 0.0
            params.append(SamplingParams(
                max_new_tokens=out_len[b], do_sample=not (greedy or top_k[b] == 1),
                temperature=temp[b], top_k=0 if greedy else top_k[b],
                top_p=1.0 if top_p[b] <= 0.0 else top_p[b], repetition_penalty=rep[b], seed=seed[b],
                eos_token_id=end_id[b], stop_sequences=stop[b] if stop else None,
                bad_words_ids=bad[b] if bad else None, logprobs=True))
            prompts.append(p)
        meta = dict(ids=ids, B=B, lens=lens, out_len=out_len, end_id=end_id, beam=beam, want_lp=want_lp, lpen=lpen,
                    div=div)
        return prompts, params, meta

    @staticmethod
    def _assemble(views, meta) -> dict:
        """``views``: per row (prompt, output, logprobs) -> FT output tensors."""
        B, lens, out_len, end_id = meta["B"], meta["lens"], meta["out_len"], meta["end_id"]
        max_total = max(lens[b] + out_len[b] for b in range(B))
        out_ids = np.full((B, 1, max_total), 0, dtype=np.int32)
        seq_len = np.zeros((B, 1), dtype=np.int32)
        cum = np.zeros((B, 1), dtype=np.float32)
        olp = np.zeros((B, 1, max(out_len)), dtype=np.float32)
        for b, (prompt, output, lps) in enumerate(views):
            toks = list(prompt) + list(output)
            out_ids[b, 0, :] = end_id[b]
            out_ids[b, 0, :len(toks)] = toks
            seq_len[b, 0] = len(toks)
            cum[b, 0] = float(np.sum(lps)) if lps else 0.0
            olp[b, 0, :len(lps)] = lps
        out = {"output_ids": out_ids, "sequence_length": seq_len}
        if meta["want_lp"]:
            out["cum_log_probs"] = cum
            out["output_log_probs"] = olp
        return out

    def infer(self, inputs: dict, request: dict, headers=None) -> dict:
        prompts, params, meta = self._prepare(inputs)
        if any(b > 1 for b in meta["beam"]):
            return self._beam_infer(meta["ids"], meta["lens"], meta["out_len"], meta["end_id"], meta["beam"],
                                    meta["lpen"], meta["div"], meta["want_lp"])
        reqs = self.generator.generate_ids(prompts, params)
        return self._assemble([(r.prompt, r.output, r.logprobs) for r in reqs], meta)

    def infer_stream(self, inputs: dict, request: dict, headers=None):
        """Decoupled (token-streaming) inference, FT's ``decoupled: True`` mode
        behind ``ModelStreamInfer``: yields the FT output tensors after every
        generation step (all rows padded to the same shapes), the last one
        complete. Beam search answers once."""
        import queue
        import threading
        prompts, params, meta = self._prepare(inputs)
        if any(b > 1 for b in meta["beam"]):
            yield self.infer(inputs, request, headers)
            return
        q: queue.Queue = queue.Queue()
        state = [(p, [], []) for p in prompts]
        lock = threading.Lock()

        def on_token(i, r):
            with lock:
                state[i] = (r.prompt, list(r.output), list(r.logprobs))
                q.put(("tok", [(a, list(b), list(c)) for a, b, c in state]))

        def run():
            try:
                reqs = self.generator.generate_ids(prompts, params, on_token=on_token)
                q.put(("done", [(r.prompt, r.output, r.logprobs) for r in reqs]))
            except Exception as e:  # noqa: BLE001 -- surfaced to the stream
                q.put(("error", e))
        threading.Thread(target=run, daemon=True).start()
        while True:
            kind, val = q.get()
            if kind == "error":
                raise val
            if kind == "done":
                yield self._assemble(val, meta)
                return
            while not q.empty():  # coalesce tokens that arrived while the consumer was busy
                nxt = q.get()
                if nxt[0] != "tok":
                    kind, val = nxt
                    break
                val = nxt[1]
            if kind == "error":
                raise val
            if kind == "done":
                yield self._assemble(val, meta)
                return
            yield self._assemble(val, meta)

    def _beam_infer(self, ids, lens, out_len, end_id, beam, lpen, div, want_lp):
        B, W = ids.shape[0], max(beam)
        max_total = max(lens[b] + out_len[b] for b in range(B))
        out_ids = np.zeros((B, W, max_total), dtype=np.int32)
        seq_len = np.zeros((B, W), dtype=np.int32)
        cum = np.zeros((B, W), dtype=np.float32)
        for b in range(B):
            p = ids[b, :lens[b]].tolist()
            res = self.generator.engine.beam_generate(p, beam[b], out_len[b], end_id[b], lpen[b], div[b],
                                                      n_return=beam[b])
            for j, (toks, c) in enumerate(zip(res.sequences, res.cum_logprobs)):
                full = p + toks
                out_ids[b, j, :] = end_id[b]
                out_ids[b, j, :len(full)] = full
                seq_len[b, j] = len(full)
                cum[b, j] = c
        out = {"output_ids": out_ids, "sequence_length": seq_len}
        if want_lp:
            out["cum_log_probs"] = cum
        return out


def main(argv=None):
    import argparse

    from .server import ModelServer
    ap = argparse.ArgumentParser()
    ap.add_argument("--model-store", default=os.getenv("MODEL_STORE", "/mnt/pvc/gptj-store/triton-model-store"))
    ap.add_argument("--http-port", type=int, default=80)
    a, rest = ap.parse_known_args(argv)
    m = FasterTransformerModel(store_dir=a.model_store)
    m.load()
    ModelServer(http_port=a.http_port, argv=rest).start([m])


def convert_main(argv=None):
    import argparse
    ap = argparse.ArgumentParser(description="HF checkpoint -> FT-style model store")
    ap.add_argument("--model-dir", required=True)
    ap.add_argument("--output-dir", required=True)
    ap.add_argument("--n-inference-gpus", "--tensor-parallelism", dest="tp", type=int, default=1)
    ap.add_argument("--data-type", default="fp16", choices=["bf16", "fp16", "fp32"])
    a = ap.parse_args(argv)
    print(write_model_store(a.model_dir, a.output_dir, a.tp, a.data_type))


if __name__ == "__main__":
    main()
