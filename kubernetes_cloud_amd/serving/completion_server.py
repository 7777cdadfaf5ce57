"""Finetune inference server (T4): ``GET /`` and ``POST /completion``.

Same CLI and request schema as finetuner-workflow/finetuner/inference.py:13-100
(``--model``, ``--device-id`` (-1 = CPU), ``--port`` 80, ``--ip``; the
``Completion`` body with prompt / max_new_tokens / temperature / top_p / top_k /
typical_p / repetition_penalty / do_sample / penalty_alpha /
num_return_sequences / stop_sequence / bad_words), the response is the
text-generation pipeline output (``[{"generated_text": ...}]``) or
``{"error": ...}``. The finetune workflow deploys it with
``--model=$INFERENCE_MODEL --port=80`` (finetune-workflow.yaml:583-619).

Differences by design: requests share one continuously batched engine (the
reference ran one HF pipeline call per request), and ``bad_words`` -- accepted
but silently dropped by the reference -- is honoured.
"""
from __future__ import annotations

from typing import List, Optional

from pydantic import BaseModel

from ..config.flags import DashParser, validation as val


class Completion(BaseModel):
    prompt: str
    max_new_tokens: Optional[int] = 10
    temperature: Optional[float] = None
    top_p: Optional[float] = None
    top_k: Optional[int] = None
    typical_p: Optional[float] = None
    repetition_penalty: Optional[float] = None
    do_sample: Optional[bool] = True
    penalty_alpha: Optional[float] = None
    num_return_sequences: Optional[int] = 1
    stop_sequence: Optional[str] = None
    bad_words: Optional[List] = None


def build_parser():
    p = DashParser(description="Text model inference HTTP server")
    p.add_argument("--model", type=str, default="distilgpt2",
                   help="Model to use for inference (directory, or HuggingFace ID) [default = distilgpt2]")
    p.add_argument("--device-id", type=val.non_negative(int, special_val=-1), default=0,
                   help="GPU ID to use for inference, or -1 for CPU [default = 0]")
    p.add_argument("--port", type=val.non_negative(int), default=80, help="Port to listen on [default = 80 (http)]")
    p.add_argument("--ip", type=str, default="0.0.0.0",
                   help="IP address to listen on [default = 0.0.0.0 (all interfaces)]")
    p.add_argument("--max-batch", type=val.positive(int), default=32,
                   help="Concurrent sequences in the engine batch [default = 32]")
    p.add_argument("--random-init", action="store_true", help="Random weights for a preset name (benchmarks)")
    return p


def create_app(generator):
    from fastapi import FastAPI
    from fastapi.middleware.cors import CORSMiddleware

    app = FastAPI(title="Inference API")
    app.add_middleware(CORSMiddleware, allow_origins=["*"], allow_methods=["*"], allow_headers=["*"])

    @app.get("/")
    def get_health():
        return "OK"

    @app.post("/completion")
    def completion(c: Completion):
        try:
            return generator(c.prompt, max_new_tokens=c.max_new_tokens, temperature=c.temperature, top_p=c.top_p,
                             top_k=c.top_k, typical_p=c.typical_p, repetition_penalty=c.repetition_penalty,
                             do_sample=c.do_sample, penalty_alpha=c.penalty_alpha,
                             num_return_sequences=c.num_return_sequences, stop_sequence=c.stop_sequence,
                             bad_words=c.bad_words)
        except Exception as e:  # noqa: BLE001 -- same contract as the reference
            return {"error": str(e)}

    return app


def main(argv=None):
    import torch
    import uvicorn

    from .text import TextGenerator, load_lm
    args = build_parser().parse_args(argv)
    dev = torch.device("cpu") if args.device_id == -1 else torch.device("cuda", args.device_id)
    model, tok = load_lm(args.model, device=dev, random_init=args.random_init)
    gen = TextGenerator(model, tok, max_slots=args.max_batch)
    uvicorn.run(create_app(gen), host=args.ip, port=args.port)


if __name__ == "__main__":
    main()
