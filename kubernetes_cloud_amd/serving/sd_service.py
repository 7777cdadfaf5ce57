"""Stable Diffusion txt2img predictor (S1) and serializer CLI (S2).

Predictor contract = online-inference/stable-diffusion/service/service.py:
31-270: ``--model-id``/``MODEL_ID``, ``--precision`` float16|float32,
``--guidance-scale``/``CONDITION_SCALE`` 7.0, ``--num-inference-steps``/
``NUM_INFERENCE_STEPS`` 50, ``--seed``/``SEED``, ``--width``/``WIDTH``,
``--height``/``HEIGHT`` 512, ``--tensorized``; KServe name = last path
component; request ``{"prompt", "parameters": {...}}`` with case-insensitive
keys; response = raw PNG bytes. Loads the diffusers layout or the tensorized
layout (``{encoder,vae,unet}.tensors``) and runs the LMS scheduler.

MI355X-first additions: bf16 compute (``--precision float16`` selects fp16),
and a dynamic micro-batcher -- concurrent requests with the same size/steps/
guidance are denoised together as one CFG batch (up to ``--max-batch``, 8 by
default = BASELINE config 5), each with its own seeded latents.

Serializer contract = serializer/serialize.py:53-75: ``--model-id``,
``--save-path``; writes the tensorized layout + tokenizer.
"""
from __future__ import annotations

import argparse
import io
import logging
import os
import queue
import threading
import time
from concurrent.futures import Future

import torch

from .server import InvalidInput, Model, ModelServer

log = logging.getLogger("kca.serving")


def get_args(argv=None):
    p = argparse.ArgumentParser()
    p.add_argument("--model-id", default=os.getenv("MODEL_ID", "/mnt/models/CompVis/stable-diffusion-v1-4"), type=str)
    p.add_argument("--precision", choices=["float16", "float32", "bfloat16"], default="float16", type=str)
    p.add_argument("--guidance-scale", default=float(os.getenv("CONDITION_SCALE", 7.0)), type=float)
    p.add_argument("--num-inference-steps", default=int(os.getenv("NUM_INFERENCE_STEPS", 50)), type=int)
    p.add_argument("--seed", default=os.getenv("SEED"), type=int)
    p.add_argument("--width", default=int(os.getenv("WIDTH", 512)), type=int)
    p.add_argument("--height", default=int(os.getenv("HEIGHT", 512)), type=int)
    p.add_argument("--tensorized", default=False, action="store_true")
    p.add_argument("--max-batch", default=int(os.getenv("MAX_BATCH", 8)), type=int)
    p.add_argument("--batch-window-ms", default=float(os.getenv("BATCH_WINDOW_MS", 5.0)), type=float)
    p.add_argument("--deterministic", default=os.getenv("DETERMINISTIC", "0") in ("1", "true", "True"),
                   action="store_true", help="bit-identical images per seed (deterministic MIOpen solvers only)")
    args, _ = p.parse_known_args(argv)
    args.model_name = args.model_id.rstrip("/").split("/")[-1]
    return args


def png_bytes(img) -> bytes:
    buf = io.BytesIO()
    img.save(buf, format="PNG")
    return buf.getvalue()


class SDPredictor(Model):
    def __init__(self, model_name: str, model_id: str, precision: str = "float16", guidance_scale: float = 7.0,
                 num_inference_steps: int = 50, seed: int | None = None, width: int = 512, height: int = 512,
                 tensorized: bool = False, max_batch: int = 8, batch_window_ms: float = 5.0, pipeline=None,
                 device=None, deterministic: bool = False, **_):
        super().__init__(model_name)
        self.model_id, self.tensorized = model_id, tensorized
        self.precision = precision
        self.parameters = {"GUIDANCE_SCALE": guidance_scale, "NUM_INFERENCE_STEPS": num_inference_steps,
                           "SEED": seed, "WIDTH": width, "HEIGHT": height}
        self.max_batch, self.window = max_batch, batch_window_ms / 1000.0
        self.expect_wait = float(os.getenv("BATCH_EXPECT_WAIT_MS", 50.0)) / 1000.0
        self.deterministic = deterministic
        self.pipeline = pipeline
        self.device = device
        self._q: queue.Queue = queue.Queue()
        self._worker = None
        if pipeline is not None:
            self.ready = True

    # ----------------------------------------------------------- loading
    def load(self):
        from ..models.sd_pipeline import StableDiffusionPipeline
        dev = self.device or (torch.device("cuda", 0) if torch.cuda.is_available() else torch.device("cpu"))
        dt = {"float16": torch.float16, "float32": torch.float32, "bfloat16": torch.bfloat16}[self.precision]
        if dev.type == "cuda" and dt == torch.float16:
            dt = torch.bfloat16  # MFMA bf16 path; fp16 UNet activations overflow without autocast
        if dev.type == "cpu":
            dt = torch.float32
        if self.deterministic:  # same seed -> bit-identical PNG (utils/miopen.py: split-K atomics otherwise)
            from ..utils import miopen
            miopen.configure(deterministic=True)
        t0 = time.perf_counter()
        if self.tensorized:
            self.pipeline = StableDiffusionPipeline.from_tensorized(self.model_id, device=dev, dtype=dt,
                                                                    scheduler="LMSDiscreteScheduler")
        else:
            self.pipeline = StableDiffusionPipeline.from_pretrained(self.model_id, device=dev, dtype=dt,
                                                                    scheduler="LMSDiscreteScheduler")
        log.info("Loaded %s in %.2fs", self.name, time.perf_counter() - t0)
        self.ready = True

    # ----------------------------------------------------------- request
    def configure_request(self, request: dict, rp: dict) -> dict:
        for k, v in (request.get("parameters") or {}).items():
            if k.upper() in rp:
                rp[k.upper()] = v
        return rp

    def _key(self, rp):
        return (int(rp["HEIGHT"]), int(rp["WIDTH"]), int(rp["NUM_INFERENCE_STEPS"]), float(rp["GUIDANCE_SCALE"]))

    def _latents(self, rp, seed):
        pipe = self.pipeline
        f = 2 ** (len(pipe.vae.config.block_out_channels) - 1)
        g = torch.Generator(device="cpu")
        if seed is None:
            g.seed()
        else:
            g.manual_seed(int(seed))
        return torch.randn(1, pipe.unet.config.in_channels, int(rp["HEIGHT"]) // f, int(rp["WIDTH"]) // f,
                           generator=g)

    def generate(self, prompts: list[str], rp: dict, seeds: list) -> list:
        lat = torch.cat([self._latents(rp, s) for s in seeds])
        with torch.no_grad():
            return self.pipeline(prompts, height=int(rp["HEIGHT"]), width=int(rp["WIDTH"]),
                                 num_inference_steps=int(rp["NUM_INFERENCE_STEPS"]),
                                 guidance_scale=float(rp["GUIDANCE_SCALE"]), latents=lat)

    def predict(self, request: dict, headers=None) -> bytes:
        if "prompt" not in request:
            raise InvalidInput("request must contain 'prompt'")
        rp = self.configure_request(request, dict(self.parameters))
        if self.max_batch <= 1:
            return png_bytes(self.generate([request["prompt"]], rp, [rp["SEED"]])[0])
        fut: Future = Future()
        self._q.put((request["prompt"], rp, fut))
        self._ensure_worker()
        # the batcher hands back the image; its PNG is encoded here, in the request's own thread: encoded
        # on the batcher thread, the batch's 8 responses left ~10-20 ms apart, the next wave of requests
        # arrived as far apart, and the 5 ms collection window split it (concurrency 8 over HTTP: 5.1 ->
        # 3.6 images/s with a 3.5 s p99 in one run)
        return png_bytes(fut.result())

    # ------------------------------------------------------ micro-batcher
    def _ensure_worker(self):
        if self._worker is None:
            self._worker = threading.Thread(target=self._loop, daemon=True, name="sd-batcher")
            self._worker.start()

    def _loop(self):
        # collection: ``window`` after the first request -- but while fewer requests wait than the last
        # batch held (its clients are likely sending their next ones: over HTTP the responses, and so the
        # next requests, arrive spread over more than the window) up to ``expect_wait`` (50 ms, ~7 % of
        # a 512 px batch); one short batch resets the expectation
        pending = []
        expect = 1
        while True:
            if not pending:
                pending.append(self._q.get())
            t0 = time.perf_counter()
            while len(pending) < 4 * self.max_batch:
                wait = self.window if len(pending) >= expect else max(self.window, self.expect_wait)
                try:
                    pending.append(self._q.get(timeout=max(0.0, t0 + wait - time.perf_counter())))
                except queue.Empty:
                    break
            key = self._key(pending[0][1])
            batch = [x for x in pending if self._key(x[1]) == key][: self.max_batch]
            pending = [x for x in pending if x not in batch]
            expect = len(batch)
            try:
                imgs = self.generate([b[0] for b in batch], batch[0][1], [b[1]["SEED"] for b in batch])
                for (_, _, fut), im in zip(batch, imgs):
                    fut.set_result(im)
            except Exception as e:  # noqa: BLE001
                for _, _, fut in batch:
                    fut.set_exception(e)


def main(argv=None):
    args = get_args(argv)
    m = SDPredictor(**vars(args))
    m.load()
    ModelServer(argv=argv).start([m])


def serialize_main(argv=None):
    from ..models.sd_pipeline import StableDiffusionPipeline, serialize_pipeline
    p = argparse.ArgumentParser()
    p.add_argument("--model-id", default="CompVis/stable-diffusion-v1-4")
    p.add_argument("--save-path", default="CompVis/stable-diffusion-v1-4")
    p.add_argument("--dtype", default=None, choices=[None, "float16", "bfloat16", "float32"])
    a = p.parse_args(argv)
    if not os.path.isdir(a.model_id):
        raise SystemExit(f"{a.model_id}: not a local diffusers directory (no network)")
    pipe = StableDiffusionPipeline.from_pretrained(a.model_id)
    dt = getattr(torch, a.dtype) if a.dtype else None
    stats = serialize_pipeline(pipe, a.save_path, dtype=dt)
    print(stats)
    return stats


if __name__ == "__main__":
    main()
