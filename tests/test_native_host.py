"""Host-side native runtime: .tensors serializer/streamer, AVX host AdamW,
C++ byte-level BPE (parity vs HF `tokenizers`) and the context packer."""
import os

import numpy as np
import pytest
import torch

from kubernetes_cloud_amd.io import native

pytestmark = pytest.mark.skipif(not native.available(), reason="libkca_host.so not built")


def test_tensors_roundtrip_module(tmp_path):
    from kubernetes_cloud_amd.io.tensors import load_into_module, load_state_dict, metadata, serialize
    from kubernetes_cloud_amd.models.causal_lm import build_model
    from kubernetes_cloud_amd.models.config import PRESETS_HF, LMConfig
    cfg = dict(PRESETS_HF["gpt-j-6b"])
    cfg.update(n_embd=64, n_layer=2, n_head=4, rotary_dim=8, vocab_size=300)
    c = LMConfig.from_hf(cfg)
    m = build_model(c, dtype=torch.bfloat16, seed=1)
    p = str(tmp_path / "gptj.tensors")
    info = serialize(m, p, metadata={"arch": "gptj"})
    assert info["tensors"] == len(m.state_dict())
    assert metadata(p)["arch"] == "gptj"
    m2 = build_model(c, dtype=torch.bfloat16, seed=2)
    st = load_into_module(m2, p, device="cpu")
    assert st["bytes"] > 0
    for (k, v), (_, v2) in zip(m.state_dict().items(), m2.state_dict().items()):
        assert torch.equal(v, v2), k
    # dtype-cast path: load bf16 file into an fp32 module
    m3 = build_model(c, dtype=torch.float32, seed=3)
    load_into_module(m3, p, device="cpu")
    assert torch.equal(m3.wte.weight.bfloat16(), m.wte.weight)
    sd = load_state_dict(p)
    assert torch.equal(sd["ln_f.weight"], m.ln_f.weight)


def test_tensors_fp16_serialize(tmp_path):
    from kubernetes_cloud_amd.io.tensors import load_state_dict, read_header, serialize
    sd = {"a": torch.randn(5, 7), "b": torch.arange(10), "c": torch.zeros(0)}
    p = str(tmp_path / "x.tensors")
    serialize(sd, p, dtype=torch.float16)
    hdr, start = read_header(p)
    assert start % 4096 == 0 and all(e["offset"] % 4096 == 0 for e in hdr["tensors"])
    out = load_state_dict(p)
    assert out["a"].dtype == torch.float16 and torch.allclose(out["a"].float(), sd["a"], atol=1e-2)
    assert torch.equal(out["b"], sd["b"]) and out["c"].numel() == 0


@pytest.mark.parametrize("level", [512, 256, 1])
def test_host_adamw_matches_reference(level):
    lib = native.load()
    if level == 512 and lib.kca_host_simd_level() < 512:
        pytest.skip("no AVX-512 on this host")
    if level == 256 and lib.kca_host_simd_level() < 256:
        pytest.skip("no AVX2")
    n = 64 * 1000 + 37
    torch.manual_seed(0)
    p = torch.randn(n)
    g = torch.randn(n)
    m = torch.zeros(n)
    v = torch.zeros(n)
    pb = torch.empty(n, dtype=torch.bfloat16)
    mask = torch.randint(0, 2, ((n + 63) // 64,), dtype=torch.uint8)
    ref = p.clone()
    rm, rv = m.clone(), v.clone()
    lr, b1, b2, eps, wd = 1e-3, 0.9, 0.999, 1e-8, 0.1
    for step in (1, 2):
        bc1, bc2 = 1 - b1 ** step, 1 - b2 ** step
        lib.kca_host_adamw(p.data_ptr(), g.data_ptr(), m.data_ptr(), v.data_ptr(), pb.data_ptr(),
                           mask.data_ptr(), n, lr, b1, b2, eps, wd, bc1, bc2, 1.0, level)
        rm.mul_(b1).add_(g, alpha=1 - b1)
        rv.mul_(b2).addcmul_(g, g, value=1 - b2)
        dmask = mask.bool().repeat_interleave(64)[:n]
        ref.mul_(torch.where(dmask, 1 - lr * wd, 1.0))
        ref.addcdiv_(rm, (rv.sqrt() / (bc2 ** 0.5)).add_(eps), value=-lr / bc1)
    assert torch.allclose(p, ref, atol=1e-6, rtol=1e-5)
    assert torch.equal(pb, p.bfloat16())


def test_bpe_parity_with_hf_tokenizers(tmp_path):
    from kubernetes_cloud_amd.data.tokenizer import NativeBPE
    from .helpers import make_tokenizer
    tok = make_tokenizer(str(tmp_path), vocab_size=400)
    bpe = NativeBPE(str(tmp_path))
    texts = ["the quick brown fox's tail\n\n  jumps   over\tthe lazy dog!!  ",
             "kubernetes 1234 cloud-native, GPUs... I'll we've they'd",
             "x  \n y", "héllo wörld — “quotes” 数字", "   ", "a\n\n\nb", ""]
    for t in texts:
        assert list(bpe.encode(t)) == tok(t, add_special_tokens=False).input_ids, repr(t)
        assert bpe.decode(bpe.encode(t)) == t


def test_dataset_tokenizer_cli_and_packing(tmp_path):
    from kubernetes_cloud_amd.data.tokenized import TokenizedDataset
    from kubernetes_cloud_amd.data.tokenizer import main
    from .helpers import make_tokenizer
    make_tokenizer(str(tmp_path / "tok"), vocab_size=400)
    docs = tmp_path / "docs"
    docs.mkdir()
    for i in range(4):
        (docs / f"{i}.txt").write_text("".join(f"the quick brown fox number {j}\r\n" for j in range(i + 2)))
    out = str(tmp_path / "d.tokens")
    assert main(["-tokenizer", str(tmp_path / "tok"), "-context", "32", "-input", str(docs), "-output", out,
                 "-boundary", "\\n", "-boundary_overlap", "-1", "-reorder", "size_ascending",
                 "-sampling", "100", "-sanitize=true", "-retokenize=true"]) == 0
    a = np.fromfile(out, dtype="<u2")
    assert a.size % 32 == 0 and a.size > 0
    ds = TokenizedDataset(out, 32, pad_token_id=0, eos_token_id=0)
    assert len(ds) == a.size // 32
    # sampling 50% keeps every other context
    out2 = str(tmp_path / "d50.tokens")
    main(["-tokenizer", str(tmp_path / "tok"), "-context", "32", "-input", str(docs), "-output", out2,
          "-sampling", "50"])
    n2 = np.fromfile(out2, dtype="<u2").size // 32
    assert n2 == (len(ds) + 1) // 2 or n2 == len(ds) // 2
