"""Diffusion noise schedules and samplers (K18 / K22 in SURVEY §2.4).

* DDPM training schedule: ``add_noise`` (x_t = sqrt(a_t) x0 + sqrt(1-a_t) eps)
  and the v-prediction target (sd-finetuner/finetuner.py:476-511);
* LMS (the txt2img predictor's sampler, service.py:166-169, 182-184), PNDM /
  PLMS (the trainer's sample() pipeline, finetuner.py:422-425), DDIM and
  Euler -- all driven by diffusers-style ``scheduler_config.json``.

All math is on [B, 4, h, w] latents in fp32; the CFG combine and the sampler
update are a handful of elementwise ops per step, captured inside the
denoise-loop HIP graph by the SD pipeline.
"""
from __future__ import annotations

import json
import math
import os

import numpy as np
import torch


def make_betas(n: int = 1000, start: float = 0.00085, end: float = 0.012,
               schedule: str = "scaled_linear") -> torch.Tensor:
    if schedule == "scaled_linear":
        return torch.linspace(start ** 0.5, end ** 0.5, n, dtype=torch.float64) ** 2
    if schedule == "linear":
        return torch.linspace(start, end, n, dtype=torch.float64)
    if schedule == "squaredcos_cap_v2":
        f = lambda t: math.cos((t + 0.008) / 1.008 * math.pi / 2) ** 2  # noqa: E731
        return torch.tensor([min(1 - f((i + 1) / n) / f(i / n), 0.999) for i in range(n)], dtype=torch.float64)
    raise ValueError(schedule)


class _Base:
    order = 1

    def __init__(self, num_train_timesteps: int = 1000, beta_start: float = 0.00085, beta_end: float = 0.012,
                 beta_schedule: str = "scaled_linear", prediction_type: str = "epsilon", steps_offset: int = 1,
                 set_alpha_to_one: bool = False, skip_prk_steps: bool = True, **_):
        self.config = dict(num_train_timesteps=num_train_timesteps, beta_start=beta_start, beta_end=beta_end,
                           beta_schedule=beta_schedule, prediction_type=prediction_type,
                           steps_offset=steps_offset, set_alpha_to_one=set_alpha_to_one,
                           skip_prk_steps=skip_prk_steps, _class_name=type(self).__name__)
        self.N = num_train_timesteps
        self.betas = make_betas(num_train_timesteps, beta_start, beta_end, beta_schedule)
        self.alphas_cumprod = torch.cumprod(1.0 - self.betas, 0)
        self.prediction_type = prediction_type
        self.steps_offset = steps_offset
        self.final_alpha = torch.tensor(1.0, dtype=torch.float64) if set_alpha_to_one else self.alphas_cumprod[0]
        self.init_noise_sigma = 1.0
        self.timesteps = torch.arange(num_train_timesteps - 1, -1, -1)

    @classmethod
    def from_config(cls, cfg: dict):
        return cls(**cfg)

    @classmethod
    def from_pretrained(cls, path: str):
        p = os.path.join(path, "scheduler_config.json")
        with open(p) as f:
            return cls.from_config(json.load(f))

    def save_pretrained(self, path: str):
        os.makedirs(path, exist_ok=True)
        with open(os.path.join(path, "scheduler_config.json"), "w") as f:
            json.dump(self.config, f, indent=2)

    # ---- training
    def _ac(self, t: torch.Tensor, like: torch.Tensor):
        a = self.alphas_cumprod.to(like.device)[t.to(like.device).long()].float()
        while a.dim() < like.dim():
            a = a[..., None]
        return a

    def add_noise(self, x0: torch.Tensor, noise: torch.Tensor, t: torch.Tensor) -> torch.Tensor:
        a = self._ac(t, x0)
        return (a.sqrt() * x0.float() + (1 - a).sqrt() * noise.float()).to(x0.dtype)

    def get_velocity(self, x0: torch.Tensor, noise: torch.Tensor, t: torch.Tensor) -> torch.Tensor:
        a = self._ac(t, x0)
        return (a.sqrt() * noise.float() - (1 - a).sqrt() * x0.float()).to(x0.dtype)

    def scale_model_input(self, x, t):
        return x

    def _inference_steps(self, n: int) -> np.ndarray:
        ratio = self.N // n
        return (np.arange(0, n) * ratio).round()[::-1].astype(np.int64) + self.steps_offset

    def _eps(self, model_out, x, a):
        if self.prediction_type == "epsilon":
            return model_out
        if self.prediction_type == "v_prediction":
            return a.sqrt() * model_out + (1 - a).sqrt() * x
        if self.prediction_type == "sample":
            return (x - a.sqrt() * model_out) / (1 - a).sqrt()
        raise ValueError(self.prediction_type)


class DDPMScheduler(_Base):
    def set_timesteps(self, n: int, device=None):
        self.timesteps = torch.from_numpy(self._inference_steps(n) - self.steps_offset).to(device)
        self._n = n

    def step(self, model_out, t, x, generator=None):
        t = int(t)
        prev = t - self.N // self._n
        a_t = self.alphas_cumprod[t].item()
        a_p = self.alphas_cumprod[prev].item() if prev >= 0 else 1.0
        b_t = 1 - a_t / a_p
        eps = self._eps(model_out.float(), x.float(), torch.tensor(a_t))
        x0 = (x.float() - math.sqrt(1 - a_t) * eps) / math.sqrt(a_t)
        mean = (math.sqrt(a_p) * b_t / (1 - a_t)) * x0 + (math.sqrt(1 - b_t) * (1 - a_p) / (1 - a_t)) * x.float()
        if prev >= 0:
            var = max((1 - a_p) / (1 - a_t) * b_t, 1e-20)
            mean = mean + math.sqrt(var) * torch.randn(x.shape, generator=generator, device=x.device)
        return mean.to(x.dtype)


class DDIMScheduler(_Base):
    def set_timesteps(self, n: int, device=None):
        self.timesteps = torch.from_numpy(self._inference_steps(n)).clamp(max=self.N - 1).to(device)
        self._n = n

    def step(self, model_out, t, x, eta: float = 0.0, generator=None):
        t = int(t)
        prev = t - self.N // self._n
        a_t = self.alphas_cumprod[t].item()
        a_p = self.alphas_cumprod[prev].item() if prev >= 0 else self.final_alpha.item()
        eps = self._eps(model_out.float(), x.float(), torch.tensor(a_t))
        x0 = (x.float() - math.sqrt(1 - a_t) * eps) / math.sqrt(a_t)
        sigma = eta * math.sqrt((1 - a_p) / (1 - a_t) * (1 - a_t / a_p))
        out = math.sqrt(a_p) * x0 + math.sqrt(max(1 - a_p - sigma ** 2, 0.0)) * eps
        if sigma > 0:
            out = out + sigma * torch.randn(x.shape, generator=generator, device=x.device)
        return out.to(x.dtype)


class PNDMScheduler(_Base):
    """PLMS (skip_prk_steps=True, the SD default) -- 4th-order linear multistep."""

    def set_timesteps(self, n: int, device=None):
        ts = self._inference_steps(n)
        # PLMS: first step repeated (diffusers: concat(ts[:-1], ts[-2:-1], ts[-1:]) reversed order)
        plms = np.concatenate([ts[:-1], ts[-2:-1], ts[-1:]])
        self.timesteps = torch.from_numpy(plms).to(device)
        self._n = n
        self.ets = []
        self.counter = 0
        self.cur_sample = None

    def _prev_sample(self, x, t, prev, eps):
        a_t = self.alphas_cumprod[t].item()
        a_p = self.alphas_cumprod[prev].item() if prev >= 0 else self.final_alpha.item()
        b_t, b_p = 1 - a_t, 1 - a_p
        coeff = (a_p / a_t) ** 0.5
        denom = a_t * b_p ** 0.5 + (a_t * b_t * a_p) ** 0.5
        return coeff * x - (a_p - a_t) * eps / denom

    def step(self, model_out, t, x, generator=None):
        t = int(t)
        prev = t - self.N // self._n
        eps = model_out.float()
        if self.prediction_type == "v_prediction":
            a = self.alphas_cumprod[t].float()
            eps = a.sqrt() * eps + (1 - a).sqrt() * x.float()
        if self.counter != 1:
            self.ets = self.ets[-3:]
            self.ets.append(eps)
        else:
            prev = t
            t = t + self.N // self._n
        if len(self.ets) == 1 and self.counter == 0:
            mo = eps
            self.cur_sample = x.float()
        elif len(self.ets) == 1 and self.counter == 1:
            mo = (eps + self.ets[-1]) / 2
            x = self.cur_sample
            self.cur_sample = None
        elif len(self.ets) == 2:
            mo = (3 * self.ets[-1] - self.ets[-2]) / 2
        elif len(self.ets) == 3:
            mo = (23 * self.ets[-1] - 16 * self.ets[-2] + 5 * self.ets[-3]) / 12
        else:
            mo = (55 * self.ets[-1] - 59 * self.ets[-2] + 37 * self.ets[-3] - 9 * self.ets[-4]) / 24
        out = self._prev_sample(x.float(), t, prev, mo)
        self.counter += 1
        return out.to(model_out.dtype)


class LMSDiscreteScheduler(_Base):
    """k-diffusion LMS (order 4) over Karras sigmas of the discrete schedule."""

    def __init__(self, *a, **k):
        super().__init__(*a, **k)
        self.sigmas_train = ((1 - self.alphas_cumprod) / self.alphas_cumprod) ** 0.5

    def set_timesteps(self, n: int, device=None):
        ts = np.linspace(0, self.N - 1, n, dtype=np.float64)[::-1].copy()
        sig = self.sigmas_train.numpy()
        s = np.interp(ts, np.arange(len(sig)), sig)
        self.sigmas = torch.from_numpy(np.concatenate([s, [0.0]])).float()
        self.timesteps = torch.from_numpy(ts).to(device)
        self.init_noise_sigma = float(self.sigmas.max())
        self.derivs = []
        self._idx = {float(t): i for i, t in enumerate(ts)}
        self._n = n

    def scale_model_input(self, x, t):
        s = self.sigmas[self._idx[float(t)]]
        return x / ((s ** 2 + 1) ** 0.5)

    def _coef(self, order, i, j):
        sig = self.sigmas.double().numpy()

        def lm(tau):
            p = 1.0
            for k in range(order):
                if j == k:
                    continue
                p *= (tau - sig[i - k]) / (sig[i - j] - sig[i - k])
            return p
        # Gauss-Legendre quadrature of the Lagrange basis over [sigma_i, sigma_{i+1}]
        xs, ws = np.polynomial.legendre.leggauss(16)
        a, b = sig[i], sig[i + 1]
        mid, half = (a + b) / 2, (b - a) / 2
        return float(sum(w * lm(mid + half * x) for x, w in zip(xs, ws)) * half)

    def step(self, model_out, t, x, order: int = 4, generator=None):
        i = self._idx[float(t)]
        s = self.sigmas[i].item()
        if self.prediction_type == "epsilon":
            x0 = x.float() - s * model_out.float()
        elif self.prediction_type == "v_prediction":
            x0 = model_out.float() * (-s / (s ** 2 + 1) ** 0.5) + x.float() / (s ** 2 + 1)
        else:
            x0 = model_out.float()
        d = (x.float() - x0) / s
        self.derivs.append(d)
        if len(self.derivs) > order:
            self.derivs.pop(0)
        o = min(i + 1, order)
        coeffs = [self._coef(o, i, j) for j in range(o)]
        out = x.float() + sum(c * dd for c, dd in zip(coeffs, reversed(self.derivs)))
        return out.to(model_out.dtype)


class EulerDiscreteScheduler(LMSDiscreteScheduler):
    def step(self, model_out, t, x, generator=None):
        i = self._idx[float(t)]
        s, s_next = self.sigmas[i].item(), self.sigmas[i + 1].item()
        if self.prediction_type == "epsilon":
            x0 = x.float() - s * model_out.float()
        else:
            x0 = model_out.float() * (-s / (s ** 2 + 1) ** 0.5) + x.float() / (s ** 2 + 1)
        d = (x.float() - x0) / s
        return (x.float() + d * (s_next - s)).to(model_out.dtype)


SCHEDULERS = {c.__name__: c for c in (DDPMScheduler, DDIMScheduler, PNDMScheduler, LMSDiscreteScheduler,
                                      EulerDiscreteScheduler)}


def load_scheduler(path_or_cfg, kind: str | None = None):
    if isinstance(path_or_cfg, dict):
        cfg = path_or_cfg
    else:
        with open(os.path.join(path_or_cfg, "scheduler_config.json")) as f:
            cfg = json.load(f)
    name = kind or cfg.get("_class_name", "PNDMScheduler")
    return SCHEDULERS[name].from_config(cfg)


def sd_scheduler_config(prediction_type: str = "epsilon") -> dict:
    return {"_class_name": "PNDMScheduler", "num_train_timesteps": 1000, "beta_start": 0.00085,
            "beta_end": 0.012, "beta_schedule": "scaled_linear", "prediction_type": prediction_type,
            "steps_offset": 1, "set_alpha_to_one": False, "skip_prk_steps": True}
