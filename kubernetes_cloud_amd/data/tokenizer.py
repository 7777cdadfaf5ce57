"""Dataset tokenizer: text files -> packed uint16 ``.tokens`` (D2 / N18).

CLI-compatible with the Go ``dataset_tokenizer`` the finetune workflow runs
(finetuner-workflow/finetune-workflow.yaml:441-454 -- Go-style single-dash
flags: ``-tokenizer -context -eot -pad -input -output -boundary
-boundary_overlap -reorder -sampling -sanitize= -retokenize=``); the BPE
encode and the context packing run in C++ (``csrc/tokenize/bpe.cpp``).

``-tokenizer`` is a model directory holding ``tokenizer.json`` (HF fast BPE)
or ``vocab.json`` + ``merges.txt``; ``gpt2`` / ``pile`` resolve through
``$KCA_TOKENIZER_DIR/{gpt2,pile}`` (no network in this environment).
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import random
import re
import sys

import numpy as np


def bytes_to_unicode() -> dict:
    """GPT-2's reversible byte -> printable-unicode map."""
    bs = list(range(ord("!"), ord("~") + 1)) + list(range(ord("¡"), ord("¬") + 1)) + \
        list(range(ord("®"), ord("ÿ") + 1))
    cs = bs[:]
    n = 0
    for b in range(256):
        if b not in bs:
            bs.append(b)
            cs.append(256 + n)
            n += 1
    return dict(zip(bs, (chr(c) for c in cs)))


def load_bpe_tables(path: str):
    """-> (vocab dict, merges list[(a, b)], added tokens dict, normalizer name).

    ``path``: a directory with ``tokenizer.json`` (HF fast BPE, e.g. the NeoX
    ``20B_tokenizer.json`` layout) or ``vocab.json`` + ``merges.txt`` (GPT-2),
    or a ``tokenizer.json`` file itself."""
    tj = path if path.endswith(".json") and os.path.isfile(path) else os.path.join(path, "tokenizer.json")
    if os.path.exists(tj):
        with open(tj, encoding="utf-8") as f:
            t = json.load(f)
        m = t["model"]
        if m.get("type") != "BPE":
            raise ValueError(f"{tj}: model type {m.get('type')} is not BPE")
        merges = [tuple(x.split(" ", 1)) if isinstance(x, str) else tuple(x) for x in m["merges"]]
        specials = {a["content"]: a["id"] for a in t.get("added_tokens", [])}
        norm = (t.get("normalizer") or {}).get("type") or ""
        return m["vocab"], merges, specials, norm
    with open(os.path.join(path, "vocab.json"), encoding="utf-8") as f:
        vocab = json.load(f)
    with open(os.path.join(path, "merges.txt"), encoding="utf-8") as f:
        lines = [ln.rstrip("\n") for ln in f if ln.strip() and not ln.startswith("#version")]
    merges = [tuple(ln.split(" ", 1)) for ln in lines]
    # GPT-2's end-of-text token is special (matched whole in text) in every HF tokenizer of it
    specials = {t: vocab[t] for t in ("<|endoftext|>",) if t in vocab}
    return vocab, merges, specials, ""


class NativeBPE:
    """Byte-level BPE encoder backed by ``kca_bpe_*``."""

    def __init__(self, path: str):
        from ..io import native
        self.vocab, merges, self.specials, self.normalizer = load_bpe_tables(path)
        if self.normalizer not in ("", "NFC", "NFKC", "NFD", "NFKD"):
            raise ValueError(f"unsupported normalizer {self.normalizer!r}")
        # added tokens split the text first, leftmost-longest (HF tokenizers' AddedVocabulary)
        self._split = re.compile("(" + "|".join(re.escape(t) for t in sorted(self.specials, key=len, reverse=True))
                                 + ")") if self.specials else None
        self.inv = {v: k for k, v in self.vocab.items()}
        for k, v in self.specials.items():
            self.inv.setdefault(v, k)
        b2u = bytes_to_unicode()
        self.u2b = {v: k for k, v in b2u.items()}
        # bytes that never occur in UTF-8 (0xC0, 0xC1, 0xF5-0xFF) may be absent (NeoX vocab): id -1
        byte_ids = (ctypes.c_int32 * 256)(*[self.vocab.get(b2u[b], -1) for b in range(256)])
        L, R, M = [], [], []
        for a, b in merges:
            if a in self.vocab and b in self.vocab and (a + b) in self.vocab:
                L.append(self.vocab[a])
                R.append(self.vocab[b])
                M.append(self.vocab[a + b])
        n = len(L)
        self._lib = native.load()
        self._h = self._lib.kca_bpe_new(byte_ids, n, (ctypes.c_int32 * n)(*L), (ctypes.c_int32 * n)(*R),
                                        (ctypes.c_int32 * n)(*M))

    def __del__(self):
        if getattr(self, "_h", None):
            self._lib.kca_bpe_free(self._h)
            self._h = None

    def token_id(self, tok: str) -> int | None:
        if tok in self.specials:
            return self.specials[tok]
        return self.vocab.get(tok)

    def _encode_plain(self, text: str) -> np.ndarray:
        if self.normalizer:
            import unicodedata
            text = unicodedata.normalize(self.normalizer, text)
        raw = text.encode("utf-8")
        cap = len(raw) + 16
        buf = (ctypes.c_int32 * cap)()
        n = self._lib.kca_bpe_encode(self._h, raw, len(raw), buf, cap)
        return np.frombuffer(buf, dtype=np.int32, count=n).copy()

    def encode(self, text: str) -> np.ndarray:
        if self._split is None:
            return self._encode_plain(text)
        parts = []
        for i, seg in enumerate(self._split.split(text)):
            if not seg:
                continue
            if i % 2:  # captured added token
                parts.append(np.array([self.specials[seg]], dtype=np.int32))
            else:
                parts.append(self._encode_plain(seg))
        return np.concatenate(parts) if parts else np.zeros(0, dtype=np.int32)

    def decode(self, ids) -> str:
        out = bytearray()
        for i in ids:
            s = self.inv.get(int(i), "")
            if s in self.specials:
                out += s.encode()
            else:
                out += bytes(self.u2b.get(c, ord("?")) for c in s)
        return out.decode("utf-8", errors="replace")


def sanitize_text(s: str) -> str:
    """Whitespace / line-ending fixes (the workflow's `sanitize` knob)."""
    s = s.replace("\r\n", "\n").replace("\r", "\n").replace(" ", " ")
    s = re.sub(r"[ \t]+\n", "\n", s)
    s = re.sub(r"\n{3,}", "\n\n", s)
    return s.strip("\n") + "\n" if s.strip() else ""


def order_files(files: list[str], how: str, seed: int = 0) -> list[str]:
    how = (how or "none").lower()
    if how == "size_ascending":
        return sorted(files, key=os.path.getsize)
    if how == "size_descending":
        return sorted(files, key=os.path.getsize, reverse=True)
    if how == "name_ascending":
        return sorted(files)
    if how == "name_descending":
        return sorted(files, reverse=True)
    if how in ("random", "shuffle"):
        f = sorted(files)
        random.Random(seed).shuffle(f)
        return f
    return files


def _unescape(s: str) -> str:
    return s.encode("utf-8").decode("unicode_escape") if "\\" in s else s


def tokenize_dataset(tokenizer: str, inputs: str, output: str, context: int = 2048, eot: str = "",
                     pad: str = "", boundary: str = "\n", boundary_index: int = -1, reorder: str = "",
                     sampling: float = 100.0, sanitize: bool = True, seed: int = 0) -> dict:
    from ..io import native
    if tokenizer in ("gpt2", "pile"):
        tokenizer = os.path.join(os.environ.get("KCA_TOKENIZER_DIR", "/models/tokenizers"), tokenizer)
    bpe = NativeBPE(tokenizer)
    eot = eot or "<|endoftext|>"
    eot_id = bpe.token_id(eot)
    if eot_id is None:
        raise ValueError(f"eot token {eot!r} not in vocabulary")
    pad_id = bpe.token_id(pad) if pad else eot_id
    if pad_id is None:
        raise ValueError(f"pad token {pad!r} not in vocabulary")
    b_ids = bpe.encode(_unescape(boundary)) if boundary else np.array([], dtype=np.int32)
    boundary_id = int(b_ids[0]) if len(b_ids) == 1 else -1
    if os.path.isdir(inputs):
        files = [os.path.join(r, f) for r, _, fs in os.walk(inputs) for f in fs
                 if not f.startswith(".") and not f.endswith(".tokens")]
    else:
        files = [inputs]
    files = order_files(files, reorder, seed)
    lib = native.load()
    pk = lib.kca_packer_new(context, boundary_id, boundary_index, pad_id, eot_id, float(sampling))
    n_tok = 0
    try:
        for fn in files:
            with open(fn, encoding="utf-8", errors="replace") as f:
                text = f.read()
            if sanitize:
                text = sanitize_text(text)
            if not text:
                continue
            ids = np.ascontiguousarray(np.append(bpe.encode(text), eot_id).astype(np.int32))
            if ids.max() > 0xFFFF:
                raise ValueError("token id exceeds uint16")
            n_tok += len(ids)
            lib.kca_packer_add(pk, ids.ctypes.data_as(ctypes.c_void_p), len(ids))
        st = (ctypes.c_longlong * 2)()
        if lib.kca_packer_write(pk, output.encode(), st) != 0:
            raise IOError(f"failed writing {output}")
    finally:
        lib.kca_packer_free(pk)
    return {"files": len(files), "tokens": n_tok, "contexts": st[0], "kept": st[1], "output": output}


def main(argv=None):
    # Go `flag` style: single-dash long flags, `-x=v` or `-x v`, bools as -x=true
    ap = argparse.ArgumentParser(prefix_chars="-", description="dataset_tokenizer (native)")
    ap.add_argument("-tokenizer", default="gpt2")
    ap.add_argument("-context", type=int, default=2048)
    ap.add_argument("-eot", default="")
    ap.add_argument("-pad", default="")
    ap.add_argument("-input", required=True)
    ap.add_argument("-output", required=True)
    ap.add_argument("-boundary", default="\\n")
    ap.add_argument("-boundary_overlap", type=int, default=-1)
    ap.add_argument("-reorder", default="")
    ap.add_argument("-sampling", type=float, default=100)
    ap.add_argument("-sanitize", default="false")
    ap.add_argument("-retokenize", default="true")
    ap.add_argument("-seed", type=int, default=0)
    a = ap.parse_args(argv)
    truthy = lambda s: str(s).lower() in ("1", "true", "t", "yes")  # noqa: E731
    if not truthy(a.retokenize) and os.path.exists(a.output):
        print(json.dumps({"output": a.output, "skipped": "exists"}))
        return 0
    r = tokenize_dataset(a.tokenizer, a.input, a.output, a.context, a.eot, a.pad, a.boundary,
                         a.boundary_overlap, a.reorder, a.sampling, truthy(a.sanitize), a.seed)
    print(json.dumps(r))
    return 0


if __name__ == "__main__":
    sys.exit(main())
