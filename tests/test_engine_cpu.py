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


# ------------------------------------------------------ paged KV / ragged prefill
@pytest.mark.parametrize("preset", ["gpt-j-6b", "bloom-560m"])
def test_paged_cache_matches_contiguous_and_recompute(preset):
    m = tiny(preset)
    prompts = [[5, 6, 7], list(range(1, 20)), [11, 12, 13, 14], [3] * 33]
    sp = SamplingParams(max_new_tokens=9, do_sample=False)
    paged = LLMEngine(m, max_slots=4, max_len=64, page_size=16).generate(prompts, sp)
    contig = LLMEngine(m, max_slots=4, max_len=64, page_size=0).generate(prompts, sp)
    for p, a, b in zip(prompts, paged, contig):
        assert a.output == b.output == greedy_recompute(m, p, 9)


def test_ragged_prefill_batches_and_matches_solo():
    m = tiny("gpt-j-6b")
    prompts = [[1, 2, 3], [4] * 9, [5, 6], list(range(7, 21)), [9] * 5, [2, 9, 4, 1]]
    sp = SamplingParams(max_new_tokens=5, do_sample=False)
    eng = LLMEngine(m, max_slots=8, max_len=48, page_size=16)
    reqs = eng.generate(prompts, sp)
    assert eng.stats["prefill_batches"] < len(set(map(len, prompts)))  # mixed lengths shared a pass
    assert eng.stats["prefill_pad_tokens"] > 0
    for p, r in zip(prompts, reqs):
        assert r.output == LLMEngine(m, max_slots=1, max_len=48).generate([p], sp)[0].output


def test_prefill_groups_bound_padding():
    from kubernetes_cloud_amd.engine.llm_engine import Request, _prefill_groups
    reqs = [Request(i, [0] * L, SamplingParams()) for i, L in enumerate([1000, 10, 990, 12, 400, 2000])]
    groups = _prefill_groups(reqs)
    assert sorted(r.rid for g in groups for r in g) == list(range(6))
    for g in groups:
        T, real = max(len(r.prompt) for r in g), sum(len(r.prompt) for r in g)
        assert T * len(g) - real <= max(0.25 * real, 256)
    assert [len(r.prompt) for r in groups[0]] == [10, 12]


def test_kv_page_budget_queues_and_returns_pages():
    m = tiny("gpt2")
    sp = SamplingParams(max_new_tokens=20, do_sample=False)
    prompts = [[1, 2, 3], [4, 5], [6, 7, 8, 9], [10], [11, 12]]
    # 2 pages of 16 tokens per request in the worst case, 4 pages total -> at most 2 requests in flight
    eng = LLMEngine(m, max_slots=4, max_len=32, page_size=16, kv_pages=4)
    reqs = [eng.add_request(p, sp) for p in prompts]
    eng.step()
    assert len(eng.running) == 2 and len(eng.waiting) == 3
    eng.run_until_done(reqs)
    solo = [LLMEngine(m, max_slots=1, max_len=32).generate([p], sp)[0].output for p in prompts]
    assert [r.output for r in reqs] == solo
    cache = eng.runner.cache
    assert cache.free_count() == 4 and eng._committed == 0 and all(x == 0 for x in cache.ref)
    small = LLMEngine(m, max_slots=2, max_len=32, page_size=16, kv_pages=1)
    too_big = small.add_request([1] * 20, SamplingParams(max_new_tokens=5))  # 2 pages > the whole cache
    ok = small.add_request([1] * 4, SamplingParams(max_new_tokens=5))
    small.run_until_done()
    assert too_big.finish_reason == "error" and ok.finish_reason == "length"


def test_fork_shares_full_pages_and_copies_tail():
    from kubernetes_cloud_amd.engine.runner import KVCache
    c = KVCache(1, 3, 2, 64, 4, "cpu", torch.float32, page_size=16)
    c.reserve(0, 40)  # 3 pages
    c.k[0][c.pages[0]] = torch.randn(3, 2, 16, 4)
    c.fork([1, 2], [0, 0], 37)
    assert c.pages[1][:2] == c.pages[2][:2] == c.pages[0][:2]  # 2 full pages shared
    assert c.pages[1][2] != c.pages[0][2] != c.pages[2][2]     # partial tail copied
    for s in (1, 2):
        assert torch.equal(dops.gather_kv(c.k[0], s, 37, c.table_h), dops.gather_kv(c.k[0], 0, 37, c.table_h))
    assert c.ref[c.pages[0][0]] == 3
    c.fork([0, 1], [1, 0], 37)  # permutation
    c.release(0), c.release(1), c.release(2)
    assert c.free_count() == c.n_pages and all(x == 0 for x in c.ref)


def test_paged_decode_ops_reference_match_contiguous():
    torch.manual_seed(0)
    H, Hkv, D, PS, L = 4, 2, 8, 16, 64
    contig_k, contig_v = torch.randn(3, Hkv, L, D), torch.randn(3, Hkv, L, D)
    pool_k, pool_v = torch.zeros(13, Hkv, PS, D), torch.zeros(13, Hkv, PS, D)
    perm = torch.randperm(12).view(3, 4)
    tbl = perm.to(torch.int32)
    for s in range(3):
        for j in range(4):
            pool_k[perm[s, j]] = contig_k[s, :, j * PS:(j + 1) * PS]
            pool_v[perm[s, j]] = contig_v[s, :, j * PS:(j + 1) * PS]
    qkv = torch.randn(3, (H + 2 * Hkv) * D)
    pos = torch.tensor([5, 40, 63], dtype=torch.int32)
    slots = torch.tensor([2, 0, 1], dtype=torch.int32)
    cos, sin = torch.randn(L, 2), torch.randn(L, 2)
    q1, q2 = qkv.clone(), qkv.clone()
    dops.decode_prep(q1, H, Hkv, D, 4, False, cos, sin, pos, slots, contig_k, contig_v)
    dops.decode_prep(q2, H, Hkv, D, 4, False, cos, sin, pos, slots, pool_k, pool_v, block_table=tbl)
    assert torch.equal(q1, q2)
    kl = pos + 1
    a = dops.decode_attention(q1, contig_k, contig_v, slots, kl, H, L)
    b = dops.decode_attention(q2, pool_k, pool_v, slots, kl, H, L, block_table=tbl)
    assert torch.allclose(a, b)


@pytest.mark.parametrize("page_size", [0, 16])
def test_beam_search_paged_equals_contiguous(page_size):
    m = tiny("gpt-j-6b")
    eng = LLMEngine(m, max_slots=4, max_len=64, page_size=page_size)
    res = eng.beam_generate([3, 1, 4, 1, 5, 9, 2, 6, 5, 3, 5, 8, 9, 7, 9, 3, 2], num_beams=3, max_new_tokens=12,
                            n_return=3)
    ref = LLMEngine(m, max_slots=4, max_len=64, page_size=0).beam_generate(
        [3, 1, 4, 1, 5, 9, 2, 6, 5, 3, 5, 8, 9, 7, 9, 3, 2], num_beams=3, max_new_tokens=12, n_return=3)
    assert res.sequences == ref.sequences
    if page_size:
        assert eng.runner.cache.free_count() == eng.runner.cache.n_pages


@pytest.mark.parametrize("preset,page", [("gpt-j-6b", 16), ("gpt2", 0), ("bloom-560m", 16), ("pythia-2.8b", 16)])
def test_chunked_prefill_bounds_the_gap_and_matches(preset, page):
    """a long prompt admitted while a stream decodes is
    prefilled in chunks of <= prefill_chunk tokens; the running stream gets a
    token every step throughout, and every output equals the unchunked run."""
    m = tiny(preset)
    g = torch.Generator().manual_seed(3)
    short = torch.randint(0, 97, (5,), generator=g).tolist()
    long = torch.randint(0, 97, (45,), generator=g).tolist()
    sp_run = SamplingParams(max_new_tokens=14, do_sample=False)
    sp_long = SamplingParams(max_new_tokens=6, do_sample=False)
    eng = LLMEngine(m, max_slots=4, max_len=64, page_size=page, prefill_chunk=8)
    r1 = eng.add_request(short, sp_run)
    eng.step()
    eng.step()
    r2 = eng.add_request(long, sp_long)
    counts = []
    while not r2.output and not r1.done:
        before = len(r1.output)
        eng.step()
        counts.append(len(r1.output) - before)
    assert len(counts) >= 45 // 8  # the 45-token prompt took several steps
    assert all(c == 1 for c in counts), counts  # ... and the running stream never skipped a step
    assert eng.stats["prefill_chunks"] >= 5
    assert eng.stats["max_step_prefill_tokens"] <= 8 or eng.stats["steps"] <= 1
    eng.run_until_done([r1, r2])
    assert r1.output == greedy_recompute(m, short, 14)
    assert r2.output == greedy_recompute(m, long, 6)
    ref = LLMEngine(m, max_slots=4, max_len=64, page_size=page).generate([long], sp_long)[0]
    assert r2.output == ref.output


def test_chunked_prefill_window_model():
    """GPT-Neo local layers: a continued chunk sees only the last `window` keys."""
    cfg = dict(PRESETS_HF.get("gpt-neo-125m", {}) or {})
    if not cfg:
        cfg = {"model_type": "gpt_neo", "vocab_size": 97, "hidden_size": 64, "num_layers": 2, "num_heads": 4,
               "attention_types": [[["global", "local"], 1]], "window_size": 8, "max_position_embeddings": 64}
    m = build_model(LMConfig.from_hf(cfg), dtype=torch.float32, seed=0)
    g = torch.Generator().manual_seed(5)
    short = torch.randint(0, 97, (4,), generator=g).tolist()
    long = torch.randint(0, 97, (30,), generator=g).tolist()
    eng = LLMEngine(m, max_slots=4, max_len=64, prefill_chunk=7)
    r1 = eng.add_request(short, SamplingParams(max_new_tokens=12, do_sample=False))
    eng.step()
    r2 = eng.add_request(long, SamplingParams(max_new_tokens=5, do_sample=False))
    eng.run_until_done([r1, r2])
    assert eng.stats["prefill_chunks"] >= 4
    assert r1.output == greedy_recompute(m, short, 12)
    assert r2.output == greedy_recompute(m, long, 5)


def test_batched_small_grad_accum_param_fed_twice(monkeypatch):
    """train/engine.py batches small gradient accumulations (kca_accum_grad_multi on the GPU); a
    parameter fed twice in one backward through the gradient sink (a fused block applied twice)
    must not get two entries in one launch. CPU emulation of the batched path: the result equals
    the per-parameter path."""
    import torch
    from kubernetes_cloud_amd.ops import grad_sink
    from kubernetes_cloud_amd.train import engine as E

    def run(defer):
        monkeypatch.setattr(E, "_DEFER_CPU", defer)
        torch.manual_seed(0)
        lin = torch.nn.Linear(8, 8).to(torch.bfloat16)
        eng = E.TrainEngine(lin, lr=0.0, zero_stage=0, grad_accum=1)
        flushes = []
        orig = eng._flush_small
        eng._flush_small = lambda: (flushes.append(len(eng._pend)), orig())[1]
        sink = grad_sink.lookup(lin.weight)
        g1 = torch.randn(8, 8).to(torch.bfloat16)
        g2 = torch.randn(8, 8).to(torch.bfloat16)
        sink(lin.weight, g1)
        sink(lin.weight, g2)
        eng._flush_small()
        out = eng.grad[eng._by_param[id(lin.weight)].offset:][:64].clone()
        eng.remove_hooks()
        return out, flushes, g1, g2

    got, flushes, g1, g2 = run(True)
    assert flushes[0] == 1  # the second entry for the same parameter flushed the first
    ref = g1.float().reshape(-1) + g2.float().reshape(-1)
    assert torch.allclose(got, ref)


def test_lookahead_to_fallback_drops_finished_requests():
    """A request finishing in the drained in-flight step must not be decoded again when the
    engine leaves lookahead (a multi-token bad word arrives): its slot is already released."""
    m = tiny("gpt-j-6b")
    sp = SamplingParams(max_new_tokens=6, do_sample=False)
    short = SamplingParams(max_new_tokens=2, do_sample=False)
    ban = SamplingParams(max_new_tokens=6, do_sample=False, bad_words_ids=[[96, 95]])
    solo = [LLMEngine(m, max_slots=1, max_len=40).generate([p], s)[0].output
            for p, s in (([3, 4], short), ([9, 8, 7], sp), ([5, 6], ban))]
    eng = LLMEngine(m, max_slots=3, max_len=40, pipeline=True)
    real = eng.runner.decode

    def checked(rows, *a, **kw):  # a released slot is -1: out of bounds in the GPU cache kernels
        assert all(r["slot"] >= 0 for r in rows), [r["slot"] for r in rows]
        return real(rows, *a, **kw)
    eng.runner.decode = checked
    b = eng.add_request([9, 8, 7], sp)  # slot 2: the row a stale slot -1 would alias
    a = eng.add_request([3, 4], short)
    eng.step()  # prefill (token 1) + lookahead launch of token 2
    c = eng.add_request([5, 6], ban)  # next step falls back; a's last token is in flight
    eng.run_until_done()
    assert [a.output, b.output, c.output] == solo
    assert a.finish_reason == "length" and eng.stats["finished"] == 3 and sorted(eng.free) == [0, 1, 2]
