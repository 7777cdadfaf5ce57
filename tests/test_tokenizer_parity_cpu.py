"""Native BPE (csrc/tokenize/bpe.cpp + data/tokenizer.py) against HF
``tokenizers`` on the reference's own vocabularies: GPT-2
(online-inference/fastertransformer/client/gpt_bpe/gpt2-{vocab.json,merges.txt})
and GPT-NeoX-20B (client/hf_tokenizer/20B_tokenizer.json: NFC normalizer,
space-run added tokens). Corpus: every markdown/text file of the reference
tree plus a Unicode stress corpus. Token ids must be identical."""
import glob
import os

import pytest

REF = "/root/reference"
GPT2 = os.path.join(REF, "online-inference/fastertransformer/client/gpt_bpe")
NEOX = os.path.join(REF, "online-inference/fastertransformer/client/hf_tokenizer/20B_tokenizer.json")

STRESS = [
    "Hello world! It's a test, isn't it? We'll see: you'd've thought they're done.",
    "Ünïcödé façade naïve café — “quotes” ‘single’ «guillemets» … ellipsis",
    "Ελληνικά κείμενο, русский текст, עברית, العربية ١٢٣ ٤٥٦, हिन्दी पाठ, ภาษาไทย",
    "日本語のテキスト、中文文本，한국어 텍스트。ＡＢＣ１２３ｶﾀｶﾅ",
    "emoji 👍🏽 👨‍👩‍👧‍👦 🇺🇸 ⚡️ and symbols ∑∫√∞ ≠ ≤ ≥ ± × ÷ ½ ¾ ² ³ Ⅻ ⅷ",
    "é combining (decomposed é), é precomposed, ﬁ ligature, Å Å",
    "tabs\tand\nnew\r\nlines  double  spaces   triple nbsp em　ideo ls",
    "    leading spaces and trailing spaces    ",
    "code: def f(x):\n    return x**2  # comment\n\n\n    \tindent",
    "numbers 3.14159 1,000,000 0x1F 1e-10 v1.2.3 2024-01-01T12:00:00Z",
    "URLs https://example.com/path?q=1&r=2#frag and emails a.b@c.io",
    "'s 't 're 've 'm 'll 'd 'S 'T ' s '' ''' don't DON'T rock'n'roll",
    "<|endoftext|>special in the middle<|endoftext|><|endoftext|>end",
    "mixed123abc 456def ghi789 ５６７ ٨٩",
    "​ zero width ‍ joiner ﻿ bom ­ soft hyphen",
    "𝔘𝔫𝔦𝔠𝔬𝔡𝔢 𝕞𝕒𝕥𝕙 𝒶𝓁𝓅𝒽𝒶 and ancient 𐌰𐌱𐌲 scripts, Georgian ქართული, Armenian Հայերեն",
    "x" * 300 + " " + "ab" * 150,
    " " * 50 + "a" + " " * 30 + "b" + "\n" * 5 + " \n \n",
]


def _corpus():
    files = sorted(glob.glob(os.path.join(REF, "**", "*.md"), recursive=True)) + \
        sorted(glob.glob(os.path.join(REF, "**", "*.txt"), recursive=True))
    texts = []
    for f in files:
        if f.endswith("merges.txt"):
            continue
        try:
            with open(f, encoding="utf-8") as fh:
                texts.append(fh.read())
        except (UnicodeDecodeError, OSError):
            pass
    return texts + STRESS


@pytest.fixture(scope="module")
def corpus():
    if not os.path.isdir(REF):
        pytest.skip("reference tree not mounted")
    return _corpus()


def _check(native, ref, corpus):
    bad = []
    for t in corpus:
        a = native.encode(t).tolist()
        b = ref.encode(t).ids
        if a != b:
            k = next((i for i, (x, y) in enumerate(zip(a, b)) if x != y), min(len(a), len(b)))
            bad.append((t[:60], k, a[max(0, k - 3):k + 3], b[max(0, k - 3):k + 3]))
    assert not bad, bad[:5]


def test_gpt2_vocab_parity(corpus):
    if not os.path.exists(os.path.join(GPT2, "gpt2-vocab.json")):
        pytest.skip("GPT-2 vocab not present")
    import shutil
    import tempfile

    from tokenizers import AddedToken, Tokenizer, decoders, models, pre_tokenizers

    from kubernetes_cloud_amd.data.tokenizer import NativeBPE
    d = tempfile.mkdtemp()
    shutil.copy(os.path.join(GPT2, "gpt2-vocab.json"), os.path.join(d, "vocab.json"))
    shutil.copy(os.path.join(GPT2, "gpt2-merges.txt"), os.path.join(d, "merges.txt"))
    ref = Tokenizer(models.BPE.from_file(os.path.join(d, "vocab.json"), os.path.join(d, "merges.txt")))
    ref.pre_tokenizer = pre_tokenizers.ByteLevel(add_prefix_space=False)
    ref.decoder = decoders.ByteLevel()
    ref.add_special_tokens([AddedToken("<|endoftext|>", special=True)])
    native = NativeBPE(d)
    assert len(corpus) > 20
    _check(native, ref, corpus)
    txt = STRESS[1]
    assert native.decode(native.encode(txt)) == txt


def test_neox_20b_tokenizer_parity(corpus):
    if not os.path.exists(NEOX):
        pytest.skip("20B tokenizer not present")
    from tokenizers import Tokenizer

    from kubernetes_cloud_amd.data.tokenizer import NativeBPE
    ref = Tokenizer.from_file(NEOX)
    native = NativeBPE(NEOX)
    assert native.normalizer == "NFC" and native.specials["  "] == 50276
    _check(native, ref, corpus)
