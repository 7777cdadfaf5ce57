"""Layer-split ("device_map") fallback (PAR-9; reference online-inference/bloom-176b/model/bloom.py:11,46):
budget parsing, in-order greedy placement, tied heads staying with the embedding,
streaming load from safetensors, and the BLOOM predictor's DEVICE_MAP switch."""
import pytest
import torch

from kubernetes_cloud_amd.parallel import layer_split as ls

from .helpers import make_model_dir


def test_parse_sizes():
    assert ls.parse_size("71GIB") == 71 * 2**30
    assert ls.parse_size("500MB") == 500 * 10**6
    assert ls.parse_size(1234) == 1234
    mm = ls.parse_max_memory("0:71GIB,1:1GB,cpu:2GIB")
    assert list(mm) == [torch.device("cuda", 0), torch.device("cuda", 1), torch.device("cpu")]
    with pytest.raises(ValueError):
        ls.parse_size("12 parsecs")


def _meta(preset, **over):
    from kubernetes_cloud_amd.models.causal_lm import CausalLM
    from kubernetes_cloud_amd.models.config import PRESETS_HF, LMConfig
    cfg = dict(PRESETS_HF[preset])
    cfg.update(over)
    with torch.device("meta"):
        return CausalLM(LMConfig.from_hf(cfg)).to(torch.bfloat16)


def test_plan_in_order_under_budgets():
    m = _meta("gpt-j-6b", n_embd=256, n_layer=6, n_head=4, rotary_dim=32, vocab_size=1000)
    blk = ls._nbytes(m.h[0], torch.bfloat16)
    emb = ls._nbytes(m.wte, torch.bfloat16)
    # device 0: embedding + 2 blocks; device 1: the rest + head
    dmap = ls.plan_device_map(m, {0: emb + 2 * blk + 10, 1: 100 * blk})
    devs = [dmap[f"h.{i}"].index for i in range(6)]
    assert devs == [0, 0, 1, 1, 1, 1] and dmap["wte"].index == 0 and dmap["lm_head"].index == 1
    assert dmap["ln_f"] == dmap["lm_head"]
    with pytest.raises(MemoryError):
        ls.plan_device_map(m, {0: blk // 2})


def test_tied_head_sits_with_embedding():
    m = _meta("bloom-560m", hidden_size=64, n_layer=4, n_head=4, vocab_size=500)
    blk = ls._nbytes(m.h[0], torch.bfloat16)
    emb = ls._nbytes(m.wte, torch.bfloat16) + ls._nbytes(m.emb_ln, torch.bfloat16)
    dmap = ls.plan_device_map(m, {0: emb + blk + 64, "cpu": 1 << 30})
    assert dmap["ln_f"] == dmap["wte"] == torch.device("cuda", 0)
    assert dmap["h.3"] == torch.device("cpu")


@pytest.mark.parametrize("preset,over", [("gpt-j-6b", dict(n_embd=64, n_layer=3, n_head=4, rotary_dim=8)),
                                         ("bloom-560m", dict(hidden_size=64, n_layer=3, n_head=4))])
def test_load_layer_split_matches_load_pretrained(tmp_path, preset, over):
    from kubernetes_cloud_amd.engine.llm_engine import LLMEngine, SamplingParams
    from kubernetes_cloud_amd.io.hf import load_pretrained
    d = make_model_dir(str(tmp_path / "m"), preset, vocab_size=128, tokenizer=False, **over)
    ref = load_pretrained(d, dtype=torch.float32)
    m = ls.load_layer_split(d, {"cpu": 1 << 30}, dtype=torch.float32)
    assert m.hf_device_map["h.0"] == "cpu"
    for (n, a), (_, b) in zip(ref.state_dict().items(), m.state_dict().items()):
        assert torch.equal(a, b), n
    ids = torch.tensor([[1, 2, 3, 4, 5]])
    with torch.no_grad():
        assert torch.equal(ref(ids), m(ids))
    sp = SamplingParams(max_new_tokens=5, do_sample=False)
    assert LLMEngine(m, max_slots=2, max_len=32).generate([[1, 2, 3]], sp)[0].output == \
        LLMEngine(ref, max_slots=2, max_len=32).generate([[1, 2, 3]], sp)[0].output


def test_bloom_predictor_device_map_switch(tmp_path, monkeypatch):
    from kubernetes_cloud_amd.serving.predictors import BloomPredictor, bloom_options
    d = make_model_dir(str(tmp_path / "bloom"), "bloom-560m", hidden_size=64, n_layer=2, n_head=4)
    o, p = bloom_options({"MODEL_PATH": d, "DEVICE_MAP": "auto", "MAX_MEMORY": "cpu:1GIB", "MAX_LENGTH": "12"})
    pred = BloomPredictor(options=o, params=p)
    pred.load()
    assert pred.generator.model.hf_device_map["h.1"] == "cpu"
    out = pred.predict({"instances": ["hello"]})
    assert len(out["predictions"]) == 1
