"""Evaluator CLI (T3): sample prompts against a (finetuned) model.

Same flags as finetuner-workflow/finetuner/evaluator.py:19-121 (``--model``,
``--trust-remote-code``, ``--tokenizer``, ``--eot``, ``--pad``, ``--cache``,
``--fp16``, ``--prompt`` | ``--prompt-file``, ``--prompt-tokens`` 200,
``--seed``, ``--prompt-samples`` 1, ``--top-k`` 16, ``--top-p`` .95,
``--temperature`` 1.0, ``--repetition-penalty`` 1.1) and the same sampling
(do_sample, bad_words = [[eos]], evaluator.py:175-219) and output format. The
model runs on the native engine (bf16 on MI355X unless --fp16 is given, which
selects fp16).
"""
from __future__ import annotations

import sys
import time

import torch

from ..config.flags import DashParser, FuzzyBoolAction, validation as val


def build_parser():
    p = DashParser(description="Simple Model Evaluator")
    p.add_argument("--model", type=str, required=True,
                   help="The model to evaluate against (directory, or HuggingFace ID)")
    p.add_argument("--trust-remote-code", action=FuzzyBoolAction, default=False,
                   help="Whether to trust remote code coming with the model")
    p.add_argument("--tokenizer", type=str, help="The tokenizer to use")
    p.add_argument("--eot", type=str, default="", help="EOT token to use")
    p.add_argument("--pad", type=str, default="", help="Pad token to use")
    p.add_argument("--cache", type=str, default="/tmp", help="HuggingFace cache location")
    p.add_argument("--fp16", action=FuzzyBoolAction, default=False, help="Force evaluation in fp16")
    p.add_argument("--prompt", type=str, help="Prompt to use")
    p.add_argument("--prompt-file", type=val.optional_extant_file, help="File containing prompts")
    p.add_argument("--prompt-tokens", type=val.non_negative(int), default=200, help="Number of tokens to generate")
    p.add_argument("--seed", type=val.at_most_32_bit(val.non_negative(int)), default=None, help="Random seed value")
    p.add_argument("--prompt-samples", type=val.non_negative(int), default=1, help="Number of samples to generate")
    p.add_argument("--top-k", type=val.non_negative(int), default=16, help="Top K to use for sampling")
    p.add_argument("--top-p", type=val.at_most_1(val.non_negative(float)), default=0.95,
                   help="Top P to use for sampling")
    p.add_argument("--temperature", type=val.positive(float), default=1.0, help="Temperature to use for sampling")
    p.add_argument("--repetition-penalty", type=val.positive(float), default=1.1,
                   help="Repetition penalty to use for sampling")
    return p


def read_prompts(parser, args) -> list[str]:
    if args.prompt and args.prompt_file:
        parser.error("Cannot specify both a prompt and a prompt file")
    if not args.prompt and not args.prompt_file:
        parser.error("Please specify either a prompt or a prompt file")
    if args.prompt_file:
        try:
            with open(args.prompt_file, "r", encoding="utf-8") as f:
                prompts = [ln.rstrip("\n").replace("\\n", "\n") for ln in f]
            prompts = [p for p in prompts if p]
        except OSError:
            parser.error(f"Provided prompt file could not be read: {args.prompt_file}")
        if not prompts:
            parser.error(f"Provided prompt file was blank: {args.prompt_file}")
        return prompts
    return [args.prompt.strip()]


def main(argv=None, out=None):
    from ..engine.generate import GenerationConfig, generate
    from ..io.hf import load_pretrained, load_tokenizer
    from ..utils.memory import MemoryUsage
    out = out or sys.stdout
    parser = build_parser()
    args = parser.parse_args(argv)
    args.tokenizer = args.tokenizer or args.model
    prompts = read_prompts(parser, args)
    dev = torch.device("cuda", 0) if torch.cuda.is_available() else torch.device("cpu")
    dtype = (torch.float16 if args.fp16 else torch.bfloat16) if dev.type == "cuda" else torch.float32
    print(MemoryUsage.now(), file=out)
    t0 = time.time()
    tok = load_tokenizer(args.tokenizer, args.eot, args.pad)
    model = load_pretrained(args.model, device=dev, dtype=dtype)
    if len(tok) > model.cfg.vocab_size:
        model.resize_token_embeddings(len(tok))
    model.eval()
    print(f"Loaded model in {time.time() - t0:.2f}s", file=out)
    print(MemoryUsage.now(), file=out)
    results = {}
    for i, prompt in enumerate(prompts):
        print("=============================", file=out)
        print("PROMPT:", prompt, file=out)
        print("UTILIZATION:", MemoryUsage.now(), file=out)
        ids = torch.tensor([tok.encode(prompt)])
        res = generate(model, ids, GenerationConfig(
            max_new_tokens=args.prompt_tokens, do_sample=True, top_k=args.top_k, top_p=args.top_p,
            temperature=args.temperature, repetition_penalty=args.repetition_penalty,
            num_return_sequences=args.prompt_samples, eos_token_id=tok.eos_token_id,
            pad_token_id=tok.pad_token_id, bad_words_ids=[[tok.eos_token_id]],
            seed=None if args.seed is None else args.seed + 7919 * i))
        texts = [tok.decode(s[:int(n)].tolist(), skip_special_tokens=False)
                 for s, n in zip(res.sequences, res.lengths)]
        results[prompt] = texts
        for t in texts:
            print("-----------------------------", file=out)
            print("RESPONSE:", t, file=out)
    return results


if __name__ == "__main__":
    main()
