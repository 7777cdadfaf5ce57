"""KServe predictors of the reference, on the native engine.

* ``BloomPredictor``      -- online-inference/bloom-176b/model/bloom.py:11-97 (env
  options MODEL_ID / MODEL_PATH / MODEL_TYPE / MODEL_DOWNLOAD_TIMEOUT and
  sampling defaults MIN_LENGTH / MAX_LENGTH / TEMPERATURE / TOP_K / TOP_P /
  REPETITION_PENALTY, case-insensitive per-request ``parameters`` override,
  ``.ready.txt`` gate). On a multi-GPU launch (WORLD_SIZE > 1) the model is
  tensor-parallel over RCCL instead of accelerate's layer split.
* ``GPTJPredictor``       -- tensorizer-isvc kserve_api.py:11-78 (model "gptj",
  ``MODEL_LOAD_TYPE=tensorizer|hf``, instances -> 50 sampled tokens) and the
  Flask variant flask_api.py:49-63 (``GET /``, ``GET /predict/<text>``).
* ``AITextGenPredictor``  -- custom-pytorch-aitextgen model.py:6-26 (``{"text",
  "length"}`` -> ``{"prediction"}``; GPT-2 1.5B).
* ``GPT2Transformer`` / ``GPT2Predictor`` -- gpt-2/transformer/transformer.py:9-20
  (BPE pre/post-processing around a token-id predictor, V1 ``signature_name``).
"""
from __future__ import annotations

import logging
import os
import re
import time

from .server import InvalidInput, Model, ModelServer
from .text import TextGenerator, load_lm

log = logging.getLogger("kca.serving")


# ---------------------------------------------------------------- BLOOM
def bloom_options(env=None) -> tuple[dict, dict]:
    env = os.environ if env is None else env
    model_id = env.get("MODEL_ID", "bigscience/bloom")
    options = {
        "MODEL_PATH": env.get("MODEL_PATH", "/mnt/pvc/bloom"),
        "MODEL_NAME": re.sub(r"[^\w-]", "-", model_id).lower(),
        "MODEL_TYPE": env.get("MODEL_TYPE", "text-generation"),
        "MODEL_DOWNLOAD_TIMEOUT": int(env.get("MODEL_DOWNLOAD_TIMEOUT", 300)),
        # layer-split fallback (bloom.py:11,46 device_map="auto" + max_memory): e.g.
        # DEVICE_MAP=auto MAX_MEMORY="0:71GIB,1:71GIB,2:71GIB,3:71GIB,4:71GIB"
        "DEVICE_MAP": env.get("DEVICE_MAP", ""),
        "MAX_MEMORY": env.get("MAX_MEMORY", ""),
    }
    params = {
        "MIN_LENGTH": int(env.get("MIN_LENGTH", 1)),
        "MAX_LENGTH": int(env.get("MAX_LENGTH", 40)),
        "TEMPERATURE": float(env.get("TEMPERATURE", 1.0)),
        "TOP_K": int(env.get("TOP_K", 50)),
        "TOP_P": float(env.get("TOP_P", 1.0)),
        "REPETITION_PENALTY": float(env.get("REPETITION_PENALTY", 1.0)),
    }
    return options, params


def default_max_memory(frac: float = 0.9) -> dict:
    """Every visible GPU at ``frac`` of its HBM (accelerate's "auto" budget)."""
    import torch
    n = torch.cuda.device_count()
    if n == 0:
        return {"cpu": 1 << 40}
    return {i: int(torch.cuda.get_device_properties(i).total_memory * frac) for i in range(n)}


def wait_for_ready_file(path: str, timeout_s: int, interval_s: float = 10.0):
    """bloom.py:79-90: poll ``{path}/.ready.txt`` (written by the downloader)."""
    ready = os.path.join(path, ".ready.txt")
    deadline = time.time() + timeout_s
    while True:
        if os.path.exists(ready):
            return True
        if time.time() >= deadline:
            raise TimeoutError(f"Download timeout {timeout_s}!")
        time.sleep(min(interval_s, max(0.0, deadline - time.time())))


class BloomPredictor(Model):
    def __init__(self, name: str | None = None, options: dict | None = None, params: dict | None = None,
                 generator: TextGenerator | None = None):
        o, p = bloom_options()
        self.options = options or o
        self.params = params or p
        super().__init__(name or self.options["MODEL_NAME"])
        self.generator = generator
        if generator is not None:
            self.ready = True

    def load(self):
        if self.options["MODEL_TYPE"] != "text-generation":
            raise ValueError(f"unsupported MODEL_TYPE {self.options['MODEL_TYPE']}")
        if self.options.get("DEVICE_MAP"):
            from ..io.hf import load_tokenizer
            from ..parallel.layer_split import load_layer_split
            model = load_layer_split(self.options["MODEL_PATH"], self.options.get("MAX_MEMORY") or default_max_memory())
            tok = load_tokenizer(self.options["MODEL_PATH"])
        else:
            model, tok = load_lm(self.options["MODEL_PATH"])
        self.generator = TextGenerator(model, tok)
        self.ready = True

    def request_params(self, request: dict) -> dict:
        rp = dict(self.params)
        for k, v in (request.get("parameters") or {}).items():
            if k.upper() in rp:
                rp[k.upper()] = v
        return rp

    def _gen_kwargs(self, request: dict) -> dict:
        if "instances" not in request:
            raise InvalidInput("request must contain 'instances'")
        rp = self.request_params(request)
        return dict(min_length=rp["MIN_LENGTH"], max_length=rp["MAX_LENGTH"], temperature=rp["TEMPERATURE"],
                    top_k=rp["TOP_K"], top_p=rp["TOP_P"], repetition_penalty=rp["REPETITION_PENALTY"])

    def predict(self, request: dict, headers=None) -> dict:
        kw = self._gen_kwargs(request)
        return {"predictions": self.generator(request["instances"], **kw)}

    async def apredict(self, request: dict, headers=None) -> dict:
        kw = self._gen_kwargs(request)
        return {"predictions": await self.generator.acall(request["instances"], **kw)}


# ----------------------------------------------------------------- GPT-J
class GPTJPredictor(Model):
    """Model "gptj"; weights from ``{MODEL_PATH}/gptj.tensors`` (tensorizer) or
    the HF files in MODEL_PATH (hf)."""

    def __init__(self, name: str = "gptj", model_path: str | None = None, load_type: str | None = None,
                 generator: TextGenerator | None = None, seed: int = 100):
        super().__init__(name)
        self.model_path = model_path or os.getenv("MODEL_PATH", "/mnt/pvc")
        self.load_type = load_type or os.getenv("MODEL_LOAD_TYPE") or "tensorizer"
        self.generator = generator
        self.seed = seed
        self.load_seconds = None
        if generator is not None:
            self.ready = True

    def load(self):
        if self.load_type not in ("tensorizer", "hf"):
            raise ValueError(f'model_load_type must be either "tensorizer" or "hf"; got {self.load_type}')
        t0 = time.perf_counter()
        tf = os.path.join(self.model_path, "gptj.tensors") if self.load_type == "tensorizer" else None
        model, tok = load_lm(self.model_path, tensors_file=tf)
        self.load_seconds = time.perf_counter() - t0
        log.info("Deserialized model in %.2fs using %s", self.load_seconds, self.load_type)
        self.generator = TextGenerator(model, tok)
        self.ready = True

    def complete(self, text: str, idx: int = 0) -> str:
        g = self.generator
        r = g.generate_ids([g.tokenizer.encode(text)], [g.sampling_params(
            0, max_new_tokens=50, do_sample=True, seed=self.seed + idx)])[0]
        return g.tokenizer.decode(r.prompt + r.output, skip_special_tokens=True)

    def _requests(self, payload: dict):
        if not isinstance(payload, dict):
            raise InvalidInput("Expected payload to be a dict")
        inputs = payload.get("instances") or ["Please input some text"]
        g = self.generator
        prompts = [g.tokenizer.encode(t) for t in inputs]
        params = [g.sampling_params(0, max_new_tokens=50, do_sample=True, seed=self.seed + i)
                  for i in range(len(prompts))]
        return prompts, params

    def _texts(self, reqs) -> dict:
        tok = self.generator.tokenizer
        return {"predictions": [tok.decode(r.prompt + r.output, skip_special_tokens=True) for r in reqs]}

    def predict(self, payload: dict, headers=None) -> dict:
        return self._texts(self.generator.generate_ids(*self._requests(payload)))

    async def apredict(self, payload: dict, headers=None) -> dict:
        return self._texts(await self.generator.agenerate_ids(*self._requests(payload)))


def create_gptj_text_app(predictor: GPTJPredictor):
    """Flask-API equivalent (flask_api.py:49-63): ``GET /`` and ``GET /predict/<text>``."""
    from fastapi import FastAPI
    from fastapi.responses import PlainTextResponse, Response
    app = FastAPI()

    @app.get("/")
    def index():
        return Response(status_code=200)

    @app.get("/predict/{text:path}")
    def predict(text: str):
        return PlainTextResponse(predictor.complete(text))

    return app


# -------------------------------------------------------------- GPT-2s
class AITextGenPredictor(Model):
    def __init__(self, name: str = "aitextgen", generator: TextGenerator | None = None):
        super().__init__(name)
        self.generator = generator
        if generator is not None:
            self.ready = True

    def load(self, model_path: str | None = None):
        path = model_path or os.getenv("MODEL_PATH", "/mnt/models/gpt2-xl")
        model, tok = load_lm(path, random_init=not os.path.isdir(path))
        self.generator = TextGenerator(model, tok)
        self.ready = True

    def predict(self, request: dict, headers=None) -> dict:
        if "text" not in request:
            raise InvalidInput("request must contain 'text'")
        out = self.generator(request["text"], max_length=int(request.get("length", 64)), do_sample=True,
                             temperature=0.7, top_k=0)
        return {"prediction": out[0]["generated_text"]}


class GPT2Predictor(Model):
    """Token-id predictor behind the GPT-2 transformer (the TF-Serving SavedModel
    role of gpt-2/service-*/gpt-s3-inferenceservice.yaml): instances of token
    ids -> predictions of continuation ids."""

    def __init__(self, name: str = "model", generator: TextGenerator | None = None, length: int = 40):
        super().__init__(name)
        self.generator, self.length = generator, length
        if generator is not None:
            self.ready = True

    def predict(self, request: dict, headers=None) -> dict:
        g = self.generator
        prompts = [list(map(int, ids)) for ids in request["instances"]]
        params = [g.sampling_params(len(p), max_new_tokens=self.length, do_sample=True, top_k=40)
                  for p in prompts]
        return {"predictions": [r.output for r in g.generate_ids(prompts, params)]}


class GPT2Transformer(Model):
    """KServe transformer: text <-> BPE ids around a predictor (transformer.py:9-20)."""

    def __init__(self, name: str, predictor_host: str | None, tokenizer, predictor: Model | None = None):
        super().__init__(name, predictor_host)
        self.tokenizer = tokenizer
        self.local = predictor
        self.ready = True

    def preprocess(self, inputs: dict, headers=None) -> dict:
        return {"signature_name": "predict",
                "instances": [self.tokenizer.encode(i) for i in inputs["instances"]]}

    def predict(self, payload, headers=None):
        if self.local is not None:
            return self.local.predict(payload)
        return super().predict(payload, headers)

    def postprocess(self, outputs: dict, headers=None) -> dict:
        return {"predictions": [self.tokenizer.decode(p) for p in outputs["predictions"]]}


# ------------------------------------------------------------------ CLIs
def bloom_main(argv=None):
    options, _ = bloom_options()
    wait_for_ready_file(options["MODEL_PATH"], options["MODEL_DOWNLOAD_TIMEOUT"])
    m = BloomPredictor()
    m.load()
    ModelServer(argv=argv).start([m])


def gptj_main(argv=None):
    m = GPTJPredictor()
    m.load()
    ModelServer(argv=argv).start([m])


def gptj_text_main(argv=None):
    import uvicorn
    m = GPTJPredictor()
    m.load()
    uvicorn.run(create_gptj_text_app(m), host="0.0.0.0", port=int(os.getenv("PORT", 8000)))


def aitextgen_main(argv=None):
    m = AITextGenPredictor()
    m.load()
    ModelServer(workers=1, argv=argv).start([m])


__all__ = ["BloomPredictor", "GPTJPredictor", "AITextGenPredictor", "GPT2Predictor", "GPT2Transformer",
           "bloom_options", "wait_for_ready_file", "create_gptj_text_app"]


def gpt2_predictor_main(argv=None):
    path = os.getenv("MODEL_PATH", "/mnt/pvc/gpt2")
    model, tok = load_lm(path, random_init=not os.path.isdir(path))
    ModelServer(argv=argv).start([GPT2Predictor(os.getenv("MODEL_NAME", "gpt-2"), TextGenerator(model, tok))])


def gpt2_transformer_main(argv=None):
    import argparse

    from ..io.hf import load_tokenizer
    ap = argparse.ArgumentParser()
    ap.add_argument("--model_name", default="model")
    ap.add_argument("--predictor_host", default=os.getenv("PREDICTOR_HOST"))
    a, rest = ap.parse_known_args(argv)
    tok = load_tokenizer(os.getenv("TOKENIZER_PATH", "/mnt/pvc/gpt2"))
    ModelServer(argv=rest).start([GPT2Transformer(a.model_name, a.predictor_host, tok)])


# ------------------------------------------------------ image classifier
class ImageClassifier(Model):
    """S11: ``{"instances": [{"b64": ...} | {"url": ...}]}`` -> ``{"predictions":
    [{"class", "score"}]}`` (image-classifier/transformer/transformer.py:25-48),
    served by our ResNet-50 directly instead of a TF-Serving Inception behind
    a transformer. Labels from ``LABELS_PATH`` (one per line) or ``class_<i>``."""

    def __init__(self, name: str = "classifier", model=None, labels: list | None = None, size: int = 224):
        super().__init__(name)
        self.model, self.labels, self.size = model, labels, size
        if model is not None:
            self.ready = True

    def load(self, weights: str | None = None):
        import torch

        from ..models.resnet import resnet50
        m = resnet50()
        w = weights or os.getenv("MODEL_PATH", "/mnt/models/resnet50_imagenet.pt")
        if os.path.exists(w):
            m.load_state_dict(torch.load(w, map_location="cpu", weights_only=True))
        dev = torch.device("cuda", 0) if torch.cuda.is_available() else torch.device("cpu")
        self.model = m.to(dev).eval()
        lp = os.getenv("LABELS_PATH", "")
        if lp and os.path.exists(lp):
            with open(lp) as f:
                self.labels = [ln.rstrip("\n") for ln in f]
        self.ready = True

    def _image(self, inst: dict):
        import base64
        import io

        import numpy as np
        import torch
        from PIL import Image
        if "b64" in inst:
            raw = base64.b64decode(inst["b64"])
        elif "url" in inst:
            import httpx
            raw = httpx.get(inst["url"], timeout=30.0).content
        else:
            raise InvalidInput("instance needs 'b64' or 'url'")
        img = Image.open(io.BytesIO(raw)).convert("RGB")
        W, H = img.size
        s = 256 / min(W, H)
        img = img.resize((max(1, round(W * s)), max(1, round(H * s))), Image.BILINEAR)
        W, H = img.size
        c = self.size
        img = img.crop(((W - c) // 2, (H - c) // 2, (W - c) // 2 + c, (H - c) // 2 + c))
        x = torch.from_numpy(np.asarray(img, dtype=np.float32) / 255.0).permute(2, 0, 1)
        mean = torch.tensor((0.485, 0.456, 0.406))[:, None, None]
        std = torch.tensor((0.229, 0.224, 0.225))[:, None, None]
        return (x - mean) / std

    def predict(self, request: dict, headers=None) -> dict:
        import torch
        xs = torch.stack([self._image(i) for i in request["instances"]])
        p = next(self.model.parameters())
        with torch.no_grad():
            probs = self.model(xs.to(p.device, p.dtype)).float().softmax(-1)
        sc, ix = probs.max(-1)
        lab = self.labels
        return {"predictions": [{"class": lab[int(i)] if lab and int(i) < len(lab) else f"class_{int(i)}",
                                 "score": float(s)} for s, i in zip(sc, ix)]}


def image_classifier_main(argv=None):
    """ISVC entrypoint of online-inference/image-classifier (deploy: image-classifier)."""
    from .server import ModelServer
    m = ImageClassifier(os.getenv("MODEL_NAME", "image-classifier"))
    m.load()
    ModelServer(argv=argv).start([m])
