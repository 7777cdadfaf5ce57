"""Model downloader (D1) -- the workflows' ``model_downloader`` step.

Go-style flags as the gpt_bpe ``model_downloader`` the reference workflows run
(finetune-workflow.yaml:338-376, sd-finetune-workflow-template.yaml:209-262):
``-model <hub id | local dir> -dest <dir> [-tokenizer-only true] [-type
diffusers]``, plus what the other reference download jobs did by hand:
``-ready`` writes ``{dest}/.ready.txt`` when complete (bloom-176b
download_model:1-64 / bloom.py:79-90 protocol), ``-tensorize gptj.tensors
[-dtype float16]`` serializes the downloaded causal LM into our ``.tensors``
format next to it (tensorizer-isvc model_download.py:7-25).

``check-tensorized -model M -out F`` is the workflow's pre-flight probe
(finetune-workflow.yaml:322-336): writes ``true`` to F when
``$TENSORIZED_BASE_URL/{model}/model.tensors`` answers 200, else ``false``.
"""
from __future__ import annotations

import argparse
import os
import shutil
import sys

TOKENIZER_FILES = ("tokenizer.json", "tokenizer_config.json", "vocab.json", "merges.txt", "special_tokens_map.json",
                   "added_tokens.json", "tokenizer.model", "config.json")


def _truthy(s) -> bool:
    return str(s).strip().lower() in ("1", "true", "t", "yes", "y")


def download(model: str, dest: str, tokenizer_only: bool = False, kind: str = "", token: str | None = None) -> str:
    os.makedirs(dest, exist_ok=True)
    if os.path.isdir(model):  # local mirror (air-gapped clusters, tests)
        for root, _, files in os.walk(model):
            rel = os.path.relpath(root, model)
            for f in files:
                if tokenizer_only and f not in TOKENIZER_FILES:
                    continue
                os.makedirs(os.path.join(dest, rel), exist_ok=True)
                shutil.copy2(os.path.join(root, f), os.path.join(dest, rel, f))
        return dest
    from huggingface_hub import snapshot_download
    allow = None
    if tokenizer_only:
        allow = list(TOKENIZER_FILES)
    elif kind == "diffusers":
        allow = ["*.json", "*.txt", "*.safetensors", "*.model", "*/*.json", "*/*.txt", "*/*.safetensors"]
    snapshot_download(model, local_dir=dest, allow_patterns=allow,
                      token=token or os.getenv("HUGGING_FACE_HUB_TOKEN"))
    return dest


def tensorize(dest: str, filename: str, dtype: str = "float16") -> str:
    import torch

    from ..io.hf import load_pretrained, serialize_causal_lm
    dt = getattr(torch, dtype)
    model = load_pretrained(dest, device="cpu", dtype=dt)
    out = os.path.join(dest, filename)
    serialize_causal_lm(model, out)  # config embedded: the URI alone rebuilds the model
    return out


def check_tensorized(model: str, base_url: str | None = None, timeout: float = 10.0) -> bool:
    from ..io.remote import PUBLIC_TENSORIZED, exists
    base = base_url or os.getenv("TENSORIZED_BASE_URL") or os.getenv("KCA_TENSORIZED_BASE", PUBLIC_TENSORIZED)
    return exists(f"{base.rstrip('/')}/{model}/model.tensors", timeout)  # offline / DNS failure == False


def main(argv=None):
    argv = list(sys.argv[1:] if argv is None else argv)
    if argv and argv[0] == "check-tensorized":
        ap = argparse.ArgumentParser(prog="downloader check-tensorized")
        ap.add_argument("-model", required=True)
        ap.add_argument("-out", default="/tmp/output.txt")
        a = ap.parse_args(argv[1:])
        ok = check_tensorized(a.model)
        with open(a.out, "w") as f:
            f.write("true" if ok else "false")
        return ok
    ap = argparse.ArgumentParser(prog="downloader")
    ap.add_argument("-model", required=True)
    ap.add_argument("-dest", required=True)
    ap.add_argument("-tokenizer-only", dest="tokenizer_only", default="false")
    ap.add_argument("-type", dest="kind", default="")
    ap.add_argument("-ready", action="store_true")
    ap.add_argument("-tensorize", default="")
    ap.add_argument("-dtype", default="float16")
    a = ap.parse_args(argv)
    download(a.model, a.dest, _truthy(a.tokenizer_only), a.kind)
    if a.tensorize:
        print(tensorize(a.dest, a.tensorize, a.dtype))
    if a.ready:
        from ..io.checkpoint import write_ready
        write_ready(a.dest)
    print(a.dest)
    return a.dest


if __name__ == "__main__":
    main()
