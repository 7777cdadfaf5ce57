"""Scheduler parity against independent derivations (diffusers is not importable here, and the
reference ships no sampler fixture). The reference builds its samplers from the SD-1.5
``scheduler_config`` (LMS for txt2img: online-inference/stable-diffusion/service/service.py:167,182;
PNDM for the finetuner's sample images: sd-finetuner-workflow/sd-finetuner/finetuner.py:422,443).
Pinned here, each against a formulation written from the published algorithm rather than from
models/schedulers.py:

* the "scaled_linear" beta schedule and the discrete sigma ladder (Karras et al. 2022, eq. 2);
* the LMS (k-diffusion) integration weights, against ``scipy.integrate.quad`` -- the integrator
  the diffusers / k-diffusion LMS uses -- instead of our Gauss-Legendre rule;
* one LMS step of order 1 as an Euler step in sigma;
* the PNDM PLMS update against the linear-multistep closed form of Liu et al. 2022 (eq. 12).
"""
import math

import numpy as np
import pytest
import torch

from kubernetes_cloud_amd.models.schedulers import (EulerDiscreteScheduler, LMSDiscreteScheduler,
                                                    PNDMScheduler, sd_scheduler_config)

scipy_integrate = pytest.importorskip("scipy.integrate")


def _alphas_cumprod_reference(n=1000, b0=0.00085, b1=0.012):
    betas = [(math.sqrt(b0) + (math.sqrt(b1) - math.sqrt(b0)) * i / (n - 1)) ** 2 for i in range(n)]
    out, acc = [], 1.0
    for b in betas:
        acc *= 1.0 - b
        out.append(acc)
    return np.array(out)


def _lms(steps=50, pred="epsilon"):
    s = LMSDiscreteScheduler.from_config(sd_scheduler_config(pred))
    s.set_timesteps(steps)
    return s


def test_scaled_linear_schedule_and_sigmas():
    s = _lms()
    ref = _alphas_cumprod_reference()
    np.testing.assert_allclose(s.alphas_cumprod.double().numpy(), ref, rtol=1e-6)
    sig_train = np.sqrt((1 - ref) / ref)
    ts = np.linspace(0, 999, 50)[::-1]
    ref_sig = np.interp(ts, np.arange(1000), sig_train)
    np.testing.assert_allclose(s.sigmas[:-1].double().numpy(), ref_sig, rtol=1e-5)
    assert float(s.sigmas[-1]) == 0.0
    np.testing.assert_allclose(s.init_noise_sigma, ref_sig.max(), rtol=1e-5)


@pytest.mark.parametrize("steps", [20, 50])
def test_lms_weights_match_adaptive_quadrature(steps):
    s = _lms(steps)
    sig = s.sigmas.double().numpy()
    for i in range(steps):
        order = min(i + 1, 4)
        for j in range(order):
            def basis(tau):
                p = 1.0
                for k in range(order):
                    if k != j:
                        p *= (tau - sig[i - k]) / (sig[i - j] - sig[i - k])
                return p
            ref = scipy_integrate.quad(basis, sig[i], sig[i + 1], epsrel=1e-10)[0]
            assert abs(s._coef(order, i, j) - ref) <= 1e-9 * max(1.0, abs(ref)), (i, j)


def test_lms_first_step_is_euler_in_sigma():
    torch.manual_seed(0)
    lms, eul = _lms(), EulerDiscreteScheduler.from_config(sd_scheduler_config())
    eul.set_timesteps(50)
    x = torch.randn(2, 4, 8, 8, dtype=torch.float64)
    eps = torch.randn_like(x)
    t = lms.timesteps[0]
    a = lms.step(eps, t, x)
    b = eul.step(eps, t, x)
    s0, s1 = float(lms.sigmas[0]), float(lms.sigmas[1])
    ref = x + eps * (s1 - s0)  # d = (x - (x - s*eps)) / s = eps
    torch.testing.assert_close(a, ref, rtol=1e-5, atol=1e-5)
    torch.testing.assert_close(b, ref, rtol=1e-5, atol=1e-5)


def test_pndm_plms_matches_closed_form():
    """After the warm-up, PLMS = the 4th-order Adams-Bashforth combination of the last four eps
    predictions fed through the DDIM-style transfer x_{t-d} = f(x_t, eps', t, t-d)."""
    torch.manual_seed(1)
    s = PNDMScheduler.from_config(sd_scheduler_config())
    s.set_timesteps(50)
    ac = s.alphas_cumprod.double()
    x = torch.randn(1, 4, 4, 4, dtype=torch.float64)
    epss = [torch.randn_like(x) for _ in range(8)]
    ts = [int(t) for t in s.timesteps[:8]]
    xs = x
    for k in range(8):
        xs = s.step(epss[k], ts[k], xs).double()
    # the eps history the last step combined (PNDM skips the second timestep's store: its first
    # two calls are the warm-up pair); the last update used eps of the last four stored calls
    hist = [epss[k] for k in (0, 2, 3, 4, 5, 6, 7)]
    e = (55 * hist[-1] - 59 * hist[-2] + 37 * hist[-3] - 9 * hist[-4]) / 24
    # recompute the last transfer from the state before it
    s2 = PNDMScheduler.from_config(sd_scheduler_config())
    s2.set_timesteps(50)
    x7 = x
    for k in range(7):
        x7 = s2.step(epss[k], ts[k], x7).double()
    t, step = ts[7], 1000 // 50
    prev = t - step
    a_t, a_p = float(ac[t]), float(ac[prev]) if prev >= 0 else float(s.final_alpha)
    ref = (a_p / a_t) ** 0.5 * x7 - (a_p - a_t) * e / (a_t * (1 - a_p) ** 0.5 + (a_t * (1 - a_t) * a_p) ** 0.5)
    torch.testing.assert_close(xs, ref, rtol=1e-6, atol=1e-6)
