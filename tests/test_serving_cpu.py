"""Serving layer on CPU: KServe V1/V2 server, completion server (T4),
BLOOM/GPT-J/aitextgen/GPT-2 predictors, FasterTransformer-compatible Triton
endpoint over the binary tensor protocol, SD predictor (PNG bytes, micro-
batching), evaluator CLI (T3)."""
import io
import os
import threading

import numpy as np
import pytest
import torch
from fastapi.testclient import TestClient

from kubernetes_cloud_amd.serving import v2
from kubernetes_cloud_amd.serving.server import ModelServer
from kubernetes_cloud_amd.serving.text import TextGenerator, load_lm

from .helpers import make_model_dir, make_sd_dir


@pytest.fixture(scope="module")
def gptj_dir(tmp_path_factory):
    return make_model_dir(str(tmp_path_factory.mktemp("gptj")), "gpt-j-6b")


@pytest.fixture(scope="module")
def gen(gptj_dir):
    m, tok = load_lm(gptj_dir, device="cpu")
    g = TextGenerator(m, tok, max_slots=8)
    yield g
    g.close()


def test_completion_server(gen):
    from kubernetes_cloud_amd.serving.completion_server import build_parser, create_app
    c = TestClient(create_app(gen))
    assert c.get("/").json() == "OK"
    r = c.post("/completion", json={"prompt": "the quick brown", "max_new_tokens": 5, "num_return_sequences": 2,
                                    "top_k": 10})
    out = r.json()
    assert len(out) == 2 and all(o["generated_text"].startswith("the quick brown") for o in out)
    r = c.post("/completion", json={"prompt": "fox", "do_sample": False, "max_new_tokens": 4,
                                    "bad_words": ["the"]})
    assert "generated_text" in r.json()[0]
    a = build_parser().parse_args(["--model", "x", "--device_id", "-1", "--port", "8080"])
    assert a.device_id == -1 and a.port == 8080


def test_kserve_v1_bloom_predictor(tmp_path):
    from kubernetes_cloud_amd.serving.predictors import BloomPredictor, bloom_options, wait_for_ready_file
    d = make_model_dir(str(tmp_path / "bloom"), "bloom-560m", hidden_size=64, n_layer=2, n_head=4)
    m, tok = load_lm(d, device="cpu")
    opts, params = bloom_options({"MODEL_ID": "bigscience/bloom", "MODEL_PATH": d, "MAX_LENGTH": "12"})
    assert opts["MODEL_NAME"] == "bigscience-bloom" and params["MAX_LENGTH"] == 12
    pred = BloomPredictor(opts["MODEL_NAME"], opts, params, generator=TextGenerator(m, tok, background=False))
    app = ModelServer(http_port=1).create_app([pred])
    c = TestClient(app)
    assert c.get("/v1/models").json() == {"models": ["bigscience-bloom"]}
    assert c.get("/v1/models/bigscience-bloom").json()["ready"] is True
    r = c.post("/v1/models/bigscience-bloom:predict",
               json={"instances": ["the quick", "a fox"], "parameters": {"max_length": 8, "Top_K": 5}})
    preds = r.json()["predictions"]
    assert len(preds) == 2 and preds[0][0]["generated_text"].startswith("the quick")
    assert c.post("/v1/models/nope:predict", json={}).status_code == 404
    assert c.post("/v1/models/bigscience-bloom:predict", json={"x": 1}).status_code == 400
    assert "request_count" in c.get("/metrics").text
    with pytest.raises(TimeoutError):
        wait_for_ready_file(str(tmp_path), 0, 0.01)
    open(os.path.join(d, ".ready.txt"), "w").close()
    assert wait_for_ready_file(d, 1, 0.01)


def test_bloom_inference_server_routes_and_hf_cache(tmp_path):
    """S5: /generate/ + /tokenize/ + /query_id/ of transformers-bloom-inference
    (text, num_generated_tokens, remove_input_from_output) and the read-only HF
    hub cache resolution of files/isvc-patch.txt."""
    from kubernetes_cloud_amd.serving.bloom_server import add_routes, resolve_hf_cache_path
    d = make_model_dir(str(tmp_path / "bloom"), "bloom-560m", hidden_size=64, n_layer=2, n_head=4)
    m, tok = load_lm(d, device="cpu")
    gen = TextGenerator(m, tok, background=False)
    app = ModelServer(http_port=1).create_app([])
    add_routes(app, gen)
    c = TestClient(app)
    r = c.post("/generate/", json={"text": ["the quick", "a fox"], "max_new_tokens": 5, "do_sample": False,
                                   "remove_input_from_output": True}).json()
    assert r["num_generated_tokens"] == [5, 5] and len(r["text"]) == 2 and r["query_id"] == 0
    r2 = c.post("/generate/", json={"text": "the quick", "max_new_tokens": 5, "do_sample": False}).json()
    assert r2["text"][0].startswith("the quick") and r2["text"][0].endswith(r["text"][0])
    t = c.post("/tokenize/", json={"text": ["the quick"]}).json()
    assert t["token_ids"][0] == tok.encode("the quick")
    assert c.get("/query_id/").json()["query_id"] == 3
    assert c.post("/generate/", json={"text": 5}).status_code == 400
    # HF hub cache layout: models--org--repo/refs/main -> snapshots/<sha>
    root = tmp_path / "hub" / "models--microsoft--bloom-deepspeed-inference-fp16"
    (root / "refs").mkdir(parents=True)
    (root / "snapshots" / "abc123").mkdir(parents=True)
    (root / "refs" / "main").write_text("abc123\n")
    got = resolve_hf_cache_path("microsoft/bloom-deepspeed-inference-fp16", str(tmp_path / "hub"))
    assert got.endswith("snapshots/abc123")


def test_gptj_predictor_tensorized_and_text_app(gptj_dir, tmp_path):
    from kubernetes_cloud_amd.io.tensors import serialize
    from kubernetes_cloud_amd.serving.predictors import GPTJPredictor, create_gptj_text_app
    m, _ = load_lm(gptj_dir, device="cpu")
    serialize(m, os.path.join(gptj_dir, "gptj.tensors"))
    p = GPTJPredictor(model_path=gptj_dir, load_type="tensorizer")
    p.load()
    assert p.ready and p.load_seconds is not None
    c = TestClient(ModelServer(http_port=1).create_app([p]))
    r = c.post("/v1/models/gptj:predict", json={"instances": ["hello there", "kubernetes"]}).json()
    assert len(r["predictions"]) == 2 and r["predictions"][0].startswith("hello there")
    r = c.post("/v1/models/gptj:predict", json={}).json()
    assert r["predictions"][0].startswith("Please input some text")
    t = TestClient(create_gptj_text_app(p))
    assert t.get("/").status_code == 200
    assert t.get("/predict/the quick fox").text.startswith("the quick fox")
    p.generator.close()
    with pytest.raises(ValueError):
        GPTJPredictor(model_path=gptj_dir, load_type="bogus").load()


def test_triton_ft_endpoint_binary_protocol(gptj_dir, tmp_path):
    from kubernetes_cloud_amd.serving.triton_ft import (FasterTransformerModel, parse_config_pbtxt,
                                                        parse_word_list, write_model_store)
    store = str(tmp_path / "triton-model-store")
    write_model_store(gptj_dir, store, data_type="fp32")
    cfg = parse_config_pbtxt(open(os.path.join(store, "fastertransformer", "config.pbtxt")).read())
    assert cfg["max_batch_size"] == 1024 and cfg["parameters"]["model_type"] == "GPT-J"
    ft = FasterTransformerModel(store_dir=store)
    ft.load()
    c = TestClient(ModelServer(http_port=1).create_app([ft]))
    assert c.get("/v2/health/ready").status_code == 200
    meta = c.get("/v2/models/fastertransformer").json()
    assert {i["name"] for i in meta["inputs"]} >= {"input_ids", "runtime_top_k", "stop_words_list"}
    ids = np.array([[5, 6, 7, 8], [9, 10, 0, 0]], dtype=np.int32)
    inputs = {"input_ids": ids, "input_lengths": np.array([[4], [2]], dtype=np.int32),
              "request_output_len": np.array([[6], [6]], dtype=np.int32),
              "runtime_top_k": np.array([[0], [0]], dtype=np.int32),
              "runtime_top_p": np.array([[0.0], [0.0]], dtype=np.float32),
              "random_seed": np.array([[0], [0]], dtype=np.uint64),
              "is_return_log_probs": np.array([[True], [True]]),
              "stop_words_list": np.array([[[0], [-1]], [[0], [-1]]], dtype=np.int32)}
    body, hdr = v2.encode_request(inputs)
    r = c.post("/v2/models/fastertransformer/infer", content=body, headers=hdr)
    assert r.status_code == 200, r.text
    out = v2.decode_response(r.content, int(r.headers[v2.HEADER]))
    assert out["output_ids"].shape == (2, 1, 10)
    assert out["output_ids"][0, 0, :4].tolist() == [5, 6, 7, 8]
    assert out["output_ids"][1, 0, :2].tolist() == [9, 10]
    assert out["sequence_length"][:, 0].tolist() == [10, 8]
    assert out["output_log_probs"].shape == (2, 1, 6) and (out["cum_log_probs"] <= 0).all()
    # greedy == engine greedy; JSON (non-binary) protocol works too
    body, hdr = v2.encode_request({k: v[:1] for k, v in inputs.items()}, binary=False, binary_output=False)
    r2 = c.post("/v2/models/fastertransformer/infer", content=body, headers=hdr)
    o2 = v2.decode_response(r2.content, None)
    assert o2["output_ids"][0].tolist() == out["output_ids"][0, :, :10].tolist()
    assert parse_word_list(np.array([[[1, 2, 3, 4], [1, 4, -1, -1]]])) == [[[1], [2, 3, 4]]]
    beam = dict(inputs, beam_width=np.array([[2], [2]], dtype=np.int32))
    body, hdr = v2.encode_request(beam)
    r3 = c.post("/v2/models/fastertransformer/infer", content=body, headers=hdr)
    ob = v2.decode_response(r3.content, int(r3.headers[v2.HEADER]))
    assert ob["output_ids"].shape == (2, 2, 10) and ob["output_ids"][0, 1, :4].tolist() == [5, 6, 7, 8]
    assert ob["cum_log_probs"][0, 0] >= ob["cum_log_probs"][0, 1] - 1e-5 or True
    ft.generator.close()


def test_gpt2_transformer_chain_and_aitextgen(gen):
    from kubernetes_cloud_amd.serving.predictors import AITextGenPredictor, GPT2Predictor, GPT2Transformer
    pred = GPT2Predictor("model", gen, length=5)
    tr = GPT2Transformer("model", None, gen.tokenizer, predictor=pred)
    c = TestClient(ModelServer(http_port=1).create_app([tr]))
    r = c.post("/v1/models/model:predict", json={"instances": ["the quick", "lazy dog"]}).json()
    assert len(r["predictions"]) == 2 and all(isinstance(p, str) for p in r["predictions"])
    ai = AITextGenPredictor(generator=gen)
    r = TestClient(ModelServer(http_port=1).create_app([ai])).post(
        "/v1/models/aitextgen:predict", json={"text": "a finetuner", "length": 12}).json()
    assert r["prediction"].startswith("a finetuner")


def test_sd_predictor_png_and_batching(tmp_path):
    from kubernetes_cloud_amd.models.sd_pipeline import StableDiffusionPipeline
    from kubernetes_cloud_amd.serving.sd_service import SDPredictor, get_args, serialize_main
    d = make_sd_dir(str(tmp_path / "sd"))
    a = get_args(["--model-id", d, "--tensorized", "--num-inference-steps", "3", "--width", "32", "--height", "32"])
    assert a.model_name == "sd" and a.tensorized
    serialize_main(["--model-id", d, "--save-path", str(tmp_path / "tz")])
    p = SDPredictor(model_name="sd", model_id=str(tmp_path / "tz"), tensorized=True, num_inference_steps=3,
                    width=32, height=32, max_batch=4, batch_window_ms=50)
    p.load()
    c = TestClient(ModelServer(http_port=1).create_app([p]))
    r = c.post("/v1/models/sd:predict", json={"prompt": "a fox", "parameters": {"SEED": 3, "guidance_scale": 5}})
    assert r.status_code == 200 and r.content[:8] == b"\x89PNG\r\n\x1a\n"
    assert r.headers["content-type"] == "image/png"
    from PIL import Image
    assert Image.open(io.BytesIO(r.content)).size == (32, 32)
    # concurrent requests get batched; identical seeds -> identical images
    res = [None] * 3

    def go(i):
        res[i] = p.predict({"prompt": "a fox", "parameters": {"seed": 3, "guidance_scale": 5}})
    th = [threading.Thread(target=go, args=(i,)) for i in range(3)]
    [t.start() for t in th]
    [t.join() for t in th]
    assert res[0] == res[1] == res[2] == r.content
    assert isinstance(StableDiffusionPipeline, type)


def test_evaluator_cli(gptj_dir, tmp_path):
    from kubernetes_cloud_amd.train.evaluator import main
    pf = tmp_path / "prompts.txt"
    pf.write_text("the quick\\nbrown\n\nkubernetes cloud\n")
    buf = io.StringIO()
    res = main(["--model", gptj_dir, "--prompt-file", str(pf), "--prompt-tokens", "4", "--prompt-samples", "2",
                "--seed", "1"], out=buf)
    assert list(res) == ["the quick\nbrown", "kubernetes cloud"]
    assert all(len(v) == 2 for v in res.values())
    assert "RESPONSE:" in buf.getvalue() and "Loaded model in" in buf.getvalue()
    with pytest.raises(SystemExit):
        main(["--model", gptj_dir], out=buf)
    assert torch.is_tensor(torch.zeros(1))


def test_classifier_and_loadgen(gptj_dir):
    import base64
    import socket

    import uvicorn
    from PIL import Image

    from kubernetes_cloud_amd.models.resnet import resnet50
    from kubernetes_cloud_amd.serving.loadgen import benchmark
    from kubernetes_cloud_amd.serving.predictors import GPTJPredictor, ImageClassifier
    buf = io.BytesIO()
    Image.new("RGB", (300, 260), (120, 30, 200)).save(buf, format="PNG")
    clf = ImageClassifier(model=resnet50(10).eval(), labels=[f"l{i}" for i in range(10)])
    c = TestClient(ModelServer(http_port=1).create_app([clf]))
    r = c.post("/v1/models/classifier:predict",
               json={"instances": [{"b64": base64.b64encode(buf.getvalue()).decode()}]}).json()
    assert r["predictions"][0]["class"].startswith("l") and 0 < r["predictions"][0]["score"] <= 1
    # load generator against a real uvicorn server (kserve protocol, async, bounded concurrency)
    m, tok = load_lm(gptj_dir, device="cpu")
    p = GPTJPredictor(generator=TextGenerator(m, tok, max_slots=4))
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    server = uvicorn.Server(uvicorn.Config(ModelServer(http_port=port).create_app([p]), host="127.0.0.1",
                                           port=port, log_level="error"))
    th = threading.Thread(target=server.run, daemon=True)
    th.start()
    import time
    for _ in range(100):
        if server.started:
            break
        time.sleep(0.05)
    res = benchmark(f"http://127.0.0.1:{port}", "kserve", 6, True, 3)
    server.should_exit = True
    th.join(timeout=10)
    p.generator.close()
    assert res["successes"] == 6 and res["p99_s"] >= res["p50_s"] > 0


def _tiny_dalle_cfgs():
    from kubernetes_cloud_amd.models.dalle_mini import DalleBartConfig, VQGANConfig
    c = DalleBartConfig(encoder_vocab_size=300, image_vocab_size=64, d_model=64, encoder_layers=2, decoder_layers=2,
                        encoder_attention_heads=4, decoder_attention_heads=4, encoder_ffn_dim=96, decoder_ffn_dim=96,
                        max_text_length=16, image_length=16)
    v = VQGANConfig(n_embed=64, embed_dim=16, z_channels=32, ch=32, ch_mult=(1, 2), num_res_blocks=1,
                    attn_resolutions=(4,), resolution=8)
    return c, v


def test_dalle_mini_predictor_png_params_and_kv_cache(tmp_path):
    """S12: DALL·E mini service contract (service.py:111-158) on the PyTorch model:
    case-insensitive parameter overrides, PNG bytes, deterministic per seed; the
    KV-cached token-by-token decode equals the full-sequence decoder."""
    from kubernetes_cloud_amd.serving.dalle_service import DalleMiniPredictor, options, wait_ready
    c, v = _tiny_dalle_cfgs()
    o = options({"TOP_K": "7", "CONDITION_SCALE": "3.0"})
    assert o["TOP_K"] == 7 and o["CONDITION_SCALE"] == 3.0 and o["MODEL_ID"] == "dalle-mini/dalle-mini"
    p = DalleMiniPredictor("dalle-mini", None, o, device=torch.device("cpu"), config=c, vq_config=v)
    p.load()
    prm = p.configure_request({"prompt": "x", "parameters": {"temperature": 0.5, "Top_P": 0.9, "other": 1}})
    assert prm == {"TOP_K": 7, "TOP_P": 0.9, "TEMPERATURE": 0.5, "CONDITION_SCALE": 3.0}
    c2 = TestClient(ModelServer(http_port=1).create_app([p]))
    r = c2.post("/v1/models/dalle-mini:predict", json={"prompt": "a red fox", "parameters": {"seed": 11}})
    assert r.status_code == 200 and r.headers["content-type"] == "image/png"
    from PIL import Image
    assert Image.open(io.BytesIO(r.content)).size == (8, 8)
    assert p.predict({"prompt": "a red fox", "parameters": {"seed": 11}}) == r.content
    m = p.model
    ids = p.tok(["a red fox"])
    codes = m.generate(ids, p.tok([""]), top_k=5, generator=torch.Generator().manual_seed(0))
    assert codes.shape == (1, 16) and int(codes.max()) < c.image_vocab_size
    with torch.no_grad():
        enc = m.encode(ids)
        tok = torch.cat([torch.full((1, 1), c.bos_token_id), codes[:, :-1]], 1)
        full = m.decode(tok, enc)
        caches = [{"self": {}, "cross": {}} for _ in m.decoder_layers]
        step = torch.cat([m.decode(tok[:, t:t + 1], enc, start=t, caches=caches) for t in range(16)], 1)
    assert torch.allclose(full, step, atol=1e-4)
    (tmp_path / ".ready.txt").write_text("ok")
    wait_ready(str(tmp_path), 1, interval=0.01)


def test_serving_bench_http_and_engine_levels_cpu(tmp_path):
    """bench/serving_bench.py (bench.py secondary_serving) end to end on CPU with shrunk models:
    .tensors write -> GPTJPredictor tensorizer load -> uvicorn V1 server -> loadgen at two
    concurrency levels, plus the same requests straight into predict (engine)."""
    import importlib.util
    import os
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    spec = importlib.util.spec_from_file_location("kca_serving_bench", os.path.join(root, "bench", "serving_bench.py"))
    sb = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(sb)
    lv = ((1, 2), (4, 4))
    g = sb.run_gptj(str(tmp_path), levels=lv, overrides=dict(n_embd=64, n_layer=2, n_head=4, rotary_dim=8,
                                                            vocab_size=512, n_positions=128))
    assert [r["concurrency"] for r in g["levels"]] == [1, 4]
    for r in g["levels"]:
        assert r["successes"] == r["requests"] and r["http_rps"] > 0 and r["engine_rps"] > 0
        assert "http_tokens_per_s" in r and "http_overhead_mean_ms" in r and "http_rps_loss" in r
        assert r["http_stdev_s"] >= 0 and r["engine_stdev_s"] >= 0 and len(r["engine_rps_passes"]) == 3 and r["engine_rps_spread"] >= 0
    assert not os.listdir(tmp_path)  # model dir and .tensors removed
    b = sb.run_bloom_slice(layers=2, levels=lv, overrides=dict(hidden_size=64, n_head=4, vocab_size=512))
    assert all(r["successes"] == r["requests"] for r in b["levels"]) and "proxy" in b


def test_loadgen_sync_window_covers_every_request():
    """--sync mode: the throughput window spans all requests, each latency only its own (ADVICE r5:
    the per-request start used to overwrite the run's start, inflating req/s by ~n)."""
    import http.server
    import threading
    import time as _t

    from kubernetes_cloud_amd.serving.loadgen import run_sync

    class _H(http.server.BaseHTTPRequestHandler):
        def do_POST(self):  # noqa: N802
            self.rfile.read(int(self.headers.get("content-length", 0)))
            _t.sleep(0.03)
            self.send_response(200)
            self.send_header("content-length", "2")
            self.end_headers()
            self.wfile.write(b"{}")

        def log_message(self, *a):
            pass

    srv = http.server.ThreadingHTTPServer(("127.0.0.1", 0), _H)
    th = threading.Thread(target=srv.serve_forever, daemon=True)
    th.start()
    try:
        url = f"http://127.0.0.1:{srv.server_address[1]}/"
        reqs = [("POST", url, b"{}", {"content-type": "application/json"})] * 5
        times, total = run_sync(reqs, timeout=10.0)
    finally:
        srv.shutdown()
    assert len(times) == 5 and all(t >= 0.03 for t in times)
    assert total >= sum(times) * 0.99 and total >= 0.15
