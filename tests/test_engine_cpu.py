"""Serving engine on CPU (fp32 reference paths): slot KV cache + decode step
match full recompute for every architecture, continuous batching is order
independent, sampling reference == HF warper semantics, stop/ban handling."""
import pytest
import torch

from kubernetes_cloud_amd.engine.generate import GenerationConfig, generate
from kubernetes_cloud_amd.engine.llm_engine import LLMEngine, SamplingParams
from kubernetes_cloud_amd.engine.sampling import top_k_top_p_filter
from kubernetes_cloud_amd.models.causal_lm import build_model
from kubernetes_cloud_amd.models.config import PRESETS_HF, LMConfig
from kubernetes_cloud_amd.ops import decode as dops

SMALL = {
    "gpt2": dict(n_embd=64, n_layer=2, n_head=4, n_positions=64),
    "gpt-j-6b": dict(n_embd=64, n_layer=2, n_head=4, rotary_dim=8, n_positions=64),
    "pythia-2.8b": dict(hidden_size=160, num_hidden_layers=2, num_attention_heads=2, intermediate_size=160,
                        max_position_embeddings=64),
    "bloom-560m": dict(hidden_size=64, n_layer=2, n_head=4),
}


def tiny(preset, vocab=97):
    cfg = dict(PRESETS_HF[preset])
    cfg.update(SMALL[preset])
    cfg.update(vocab_size=vocab)
    return build_model(LMConfig.from_hf(cfg), dtype=torch.float32, seed=0)


def greedy_recompute(model, prompt, n):
    ids = list(prompt)
    for _ in range(n):
        with torch.no_grad():
            lg = model(torch.tensor([ids]))[0, -1]
        ids.append(int(lg.argmax()))
    return ids[len(prompt):]


@pytest.mark.parametrize("preset", list(SMALL))
def test_engine_greedy_matches_recompute(preset):
    torch.manual_seed(0)
    m = tiny(preset)
    eng = LLMEngine(m, max_slots=4, max_len=48)
    prompts = [[5, 6, 7], [1, 2, 3, 4, 5, 6, 7, 8, 9], [11, 12, 13]]
    reqs = eng.generate(prompts, SamplingParams(max_new_tokens=8, do_sample=False))
    for p, r in zip(prompts, reqs):
        assert r.output == greedy_recompute(m, p, 8), preset
        assert r.finish_reason == "length"


def test_continuous_batching_order_independent():
    m = tiny("gpt-j-6b")
    sp = SamplingParams(max_new_tokens=6, do_sample=False)
    solo = [LLMEngine(m, max_slots=1, max_len=40).generate([p], sp)[0].output
            for p in ([3, 4], [9, 8, 7, 6, 5], [1])]
    eng = LLMEngine(m, max_slots=2, max_len=40)  # fewer slots than requests -> queueing
    a = eng.add_request([3, 4], sp)
    eng.step()
    b = eng.add_request([9, 8, 7, 6, 5], sp)
    c = eng.add_request([1], sp)
    eng.run_until_done()
    assert [a.output, b.output, c.output] == solo
    assert eng.stats["finished"] == 3 and len(eng.free) == 2


def test_sampling_seeded_and_stops():
    m = tiny("gpt2")
    eng = LLMEngine(m, max_slots=4, max_len=40)
    sp = SamplingParams(max_new_tokens=10, temperature=0.8, top_k=20, top_p=0.9, seed=1234, logprobs=True)
    r1, r2 = eng.generate([[1, 2, 3], [1, 2, 3]], sp)
    assert r1.output == r2.output and len(r1.logprobs) == 10
    assert all(lp <= 0 for lp in r1.logprobs)
    # stop sequence ends generation right after it appears
    first = r1.output[:2]
    r3 = eng.generate([[1, 2, 3]], SamplingParams(**{**sp.__dict__, "stop_sequences": [first]}))[0]
    assert r3.output == first and r3.finish_reason == "stop"
    # banning the greedy token changes the choice; eos with min_new_tokens is deferred
    g = eng.generate([[4, 5]], SamplingParams(max_new_tokens=1, do_sample=False))[0].output[0]
    nb = eng.generate([[4, 5]], SamplingParams(max_new_tokens=1, do_sample=False, bad_words_ids=[[g]]))[0]
    assert nb.output[0] != g
    e = eng.generate([[4, 5]], SamplingParams(max_new_tokens=3, do_sample=False, eos_token_id=g,
                                              min_new_tokens=2))[0]
    assert e.output[0] != g and e.output[1] != g


def test_generate_api_shapes():
    m = tiny("pythia-2.8b")
    res = generate(m, torch.tensor([[1, 2, 3]]), GenerationConfig(max_new_tokens=5, num_return_sequences=3,
                                                                  seed=0, return_logprobs=True))
    assert res.sequences.shape == (3, 8) and res.logprobs.shape == (3, 5)
    assert (res.lengths == 8).all() and res.prompt_len == 3


def test_keep_mask_matches_hf_warpers():
    torch.manual_seed(0)
    for _ in range(20):
        x = torch.randn(300) * 3
        for k, p in ((0, 0.9), (10, 1.0), (40, 0.7), (5, 0.5)):
            keep = dops.keep_mask_reference(x, k, p)
            hf = torch.isfinite(top_k_top_p_filter(x[None], k, p))[0]
            assert torch.equal(keep, hf)


def test_decode_reference_ops():
    torch.manual_seed(0)
    B, H, Hkv, D, L = 3, 4, 2, 16, 20
    kc = torch.randn(5, Hkv, L, D)
    vc = torch.randn(5, Hkv, L, D)
    q = torch.randn(B, (H + 2 * Hkv) * D)
    slots = torch.tensor([4, 0, 2], dtype=torch.int32)
    lens = torch.tensor([20, 1, 7], dtype=torch.int32)
    o = dops.decode_attention(q, kc, vc, slots, lens, H, 20)
    for b in range(B):
        s, n = int(slots[b]), int(lens[b])
        qb = q[b, :H * D].view(H, D)
        kb = kc[s, :, :n].repeat_interleave(2, 0)
        ref = torch.einsum("hn,hnd->hd", (torch.einsum("hd,hnd->hn", qb, kb) / D ** 0.5).softmax(-1),
                           vc[s, :, :n].repeat_interleave(2, 0))
        assert torch.allclose(o[b].view(H, D), ref, atol=1e-5)


def test_beam_search_matches_exhaustive():
    """W=vocab beams over 2 steps == exhaustive best 2-token continuation."""
    import itertools
    m = tiny("gpt2", vocab=11)
    eng = LLMEngine(m, max_slots=24, max_len=32)
    prompt = [1, 2, 3]
    res = eng.beam_generate(prompt, 11, 2, eos_token_id=None, len_penalty=0.0)
    best, best_s = None, -1e9
    with torch.no_grad():
        for a, b in itertools.product(range(11), range(11)):
            lp = torch.log_softmax(m(torch.tensor([prompt + [a]]))[0, -2:].float(), -1)
            s = float(lp[0, a] + lp[1, b])
            if s > best_s:
                best, best_s = [a, b], s
    assert res.sequences[0] == best and abs(res.cum_logprobs[0] - best_s) < 1e-4
    # W=1 beam == greedy; slots are returned
    g = eng.generate([prompt], SamplingParams(max_new_tokens=5, do_sample=False))[0].output
    assert eng.beam_generate(prompt, 1, 5).sequences[0] == g
    assert len(eng.free) == 24
