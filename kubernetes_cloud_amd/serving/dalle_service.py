"""DALL·E mini / mega InferenceService predictor (S12).

Same contract as the reference service
(online-inference/dalle-mini/model/service.py): env ``MODEL_ID``
(``dalle-mini/dalle-mini`` | ``dalle-mini/dalle-mega``), ``MODEL_CACHE``,
``MODEL_DOWNLOAD_TIMEOUT`` and the default generation knobs ``TOP_K`` (50),
``TOP_P`` (1.0), ``TEMPERATURE`` (1.0), ``CONDITION_SCALE`` (10.0)
(:23-46); a request ``{"prompt": str, "parameters": {...}}`` whose parameter
names override those defaults case-insensitively (:111-119); the response is
the PNG bytes of one 256x256 image (:146-158); startup waits for the
downloader's ``.ready.txt`` (:160-171). Generation and VQGAN decoding run on
``models/dalle_mini.py`` (PyTorch + this framework's kernels) instead of
JAX ``pmap``; with several local GPUs each replica pins one (KServe scales
replicas, PAR-11).
"""
from __future__ import annotations

import io
import logging
import os
import random
import time

import torch

from .server import Model, ModelServer, parse_server_args

logger = logging.getLogger("dalle")

DEFAULTS = {"TOP_K": 50, "TOP_P": 1.0, "TEMPERATURE": 1.0, "CONDITION_SCALE": 10.0}


def options(env=None) -> dict:
    env = os.environ if env is None else env
    o = {"MODEL_ID": env.get("MODEL_ID", "dalle-mini/dalle-mini"),
         "MODEL_CACHE": env.get("MODEL_CACHE", "/model-cache"),
         "MODEL_DOWNLOAD_TIMEOUT": int(env.get("MODEL_DOWNLOAD_TIMEOUT", 300))}
    for k, v in DEFAULTS.items():
        o[k] = type(v)(env.get(k, v))
    return o


class _ByteTokenizer:
    """Deterministic stand-in when the model directory ships no tokenizer files
    (random-init runs): UTF-8 bytes offset past the special ids, BOS/EOS/pad."""

    def __init__(self, vocab: int, max_len: int):
        self.vocab, self.max_len = vocab, max_len

    def __call__(self, texts):
        rows = []
        for t in texts:
            ids = [0] + [3 + b % (self.vocab - 3) for b in t.lower().encode()][: self.max_len - 2] + [2]
            rows.append(ids + [1] * (self.max_len - len(ids)))
        return torch.tensor(rows, dtype=torch.long)


class DalleMiniPredictor(Model):
    def __init__(self, name: str, model_path: str | None, opts: dict | None = None, device=None,
                 dtype=None, config=None, vq_config=None):
        super().__init__(name)
        self.model_path = model_path
        self.opts = opts or options()
        self.device = device or (torch.device("cuda", 0) if torch.cuda.is_available() else torch.device("cpu"))
        self.dtype = dtype or (torch.bfloat16 if self.device.type == "cuda" else torch.float32)
        self.config, self.vq_config = config, vq_config
        self.model = self.vqgan = self.tok = None

    def load(self):
        from ..models.dalle_mini import load_dalle
        logger.info("loading %s from %s", self.name, self.model_path)
        self.model, self.vqgan = load_dalle(self.model_path, self.device, self.dtype, self.config, self.vq_config)
        c = self.model.config
        self.tok = None
        if self.model_path and os.path.exists(os.path.join(self.model_path, "tokenizer_config.json")):
            from transformers import AutoTokenizer
            hf = AutoTokenizer.from_pretrained(self.model_path, local_files_only=True)
            self.tok = lambda texts: hf(texts, padding="max_length", truncation=True, max_length=c.max_text_length,
                                        return_tensors="pt").input_ids
        if self.tok is None:
            self.tok = _ByteTokenizer(c.encoder_vocab_size, c.max_text_length)
        self.ready = True
        return True

    def configure_request(self, request: dict) -> dict:
        p = {k: self.opts[k] for k in DEFAULTS}
        for k, v in (request.get("parameters") or {}).items():
            if k.upper() in p:
                p[k.upper()] = type(DEFAULTS[k.upper()])(v)
        return p

    @torch.no_grad()
    def generate_images(self, prompts: list[str], params: dict, seed: int | None = None) -> torch.Tensor:
        seed = random.randint(0, 2 ** 32 - 1) if seed is None else seed
        g = torch.Generator(device=self.device).manual_seed(seed)
        ids = self.tok(prompts).to(self.device)
        uncond = self.tok([""] * len(prompts)).to(self.device)
        codes = self.model.generate(ids, uncond, top_k=int(params["TOP_K"]), top_p=float(params["TOP_P"]),
                                    temperature=float(params["TEMPERATURE"]),
                                    condition_scale=float(params["CONDITION_SCALE"]), generator=g)
        return self.vqgan.decode_code(codes)

    def predict(self, request: dict, headers=None):
        params = self.configure_request(request)
        seed = request.get("parameters", {}).get("seed") if isinstance(request.get("parameters"), dict) else None
        img = self.generate_images([request["prompt"]], params, seed=seed)[0]
        from PIL import Image
        arr = (img.permute(1, 2, 0).float().cpu().numpy() * 255).astype("uint8")
        buf = io.BytesIO()
        Image.fromarray(arr).save(buf, format="PNG")
        return buf.getvalue()


def wait_ready(model_path: str, timeout_s: int, interval: float = 10.0):
    """service.py:160-171: poll for the downloader's .ready.txt."""
    ready = os.path.join(model_path, ".ready.txt")
    for _ in range(max(1, int(timeout_s // interval))):
        if os.path.exists(ready):
            return
        time.sleep(interval)
    if not os.path.exists(ready):
        raise TimeoutError(f"Download timeout {timeout_s}!")


def main(argv=None):
    o = options()
    name = o["MODEL_ID"].split("/")[-1]
    path = os.path.join(o["MODEL_CACHE"], o["MODEL_ID"])
    wait_ready(path, o["MODEL_DOWNLOAD_TIMEOUT"])
    m = DalleMiniPredictor(name, path, o)
    m.load()
    args = parse_server_args(argv)
    ModelServer(http_port=args.http_port).start([m])


if __name__ == "__main__":
    main()
