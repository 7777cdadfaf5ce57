"""MIOpen convolution-solver policy for the SD UNet / VAE (K15 convolutions).

PyTorch-ROCm asks MIOpen to *find* a solver for every new convolution config.
For the channels-last (NHWC) bf16 convolutions that search also times MIOpen's
reference "naive" direct-convolution solvers, which take seconds per call at
SD-1.5 shapes: a cold UNet training step spent > 3 minutes searching on an
MI355X, and with the naive solvers excluded it takes 5 s (they never win the
search; `MIOPEN_FIND_MODE=FAST` instead picks kernels 4-5x slower). This
matters for the KServe cold start the reference budgets
(online-inference/README.md:14,33) as much as for the finetuner.

Tuned solver parameters ship in ``tuning/miopen/``: MIOpen's user perf-db
(``*.udb.txt``, tuned igemm / CK tile parameters per conv config) and find-db
(``*.ufdb.txt``) for the SD-1.5 UNet at the bench shapes (txt2img batch 8 + CFG,
DreamBooth 8 + 8 fwd/bwd/wrw) and the VAE decoder, produced on an MI355X by
``MIOPEN_FIND_ENFORCE=3`` runs of ``bench/sd_bench.py --mode train`` and
``tools/sd_breakdown.py`` (the recipe is ``tools/miopen_tune.sh``).
Measured with vs without: UNet CFG step 34.7 -> 30.5 ms, VAE decode
52.3 -> 39.0 ms, DreamBooth 81.5 -> 92.5 samples/s. Other shapes fall back
to MIOpen's normal find, and their results are appended to the same db.

``configure()`` runs before the first convolution; explicit environment
settings win.

Determinism: for some configs MIOpen's find picks a split-K igemm kernel that
accumulates through fp32 atomics (igemm_fwd_gtcx35_nhwc_* after a zero-fill of
its workspace), so two identical calls can differ in the last bf16 bit
(measured on the tiny test UNet with ``tools/sd_determinism.py``).
``configure(deterministic=True)`` switches that solver family off (forward,
backward-data and weight-gradient GTC NHWC igemm; the CK implicit-GEMM solvers
that remain write their tiles once) and lets the naive solvers back in as the
fallback for configs nothing else covers; its find results go to a separate
user db so the tuned one keeps the fastest solvers. It must run before the
first convolution of the process. (``torch.backends.cudnn.deterministic``
itself is no use here: MIOpen then found no solver for the small-channel
``conv_in`` of the SD UNet.)
"""
from __future__ import annotations

import os

_NAIVE = ("MIOPEN_DEBUG_CONV_DIRECT_NAIVE_CONV_FWD", "MIOPEN_DEBUG_CONV_DIRECT_NAIVE_CONV_BWD",
          "MIOPEN_DEBUG_CONV_DIRECT_NAIVE_CONV_WRW")


TUNED_DB = os.path.join(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))),
                        "tuning", "miopen")


_GTC = ("MIOPEN_DEBUG_CONV_IMPLICIT_GEMM_ASM_FWD_GTC_XDLOPS_NHWC",
        "MIOPEN_DEBUG_CONV_IMPLICIT_GEMM_ASM_BWD_GTC_XDLOPS_NHWC",
        "MIOPEN_DEBUG_CONV_IMPLICIT_GEMM_ASM_WRW_GTC_XDLOPS_NHWC")
_OURS: set = set()


def configure(deterministic: bool = False) -> None:
    for k in _NAIVE:
        if k not in os.environ:
            os.environ[k] = "0"
            _OURS.add(k)
        if deterministic and k in _OURS:
            os.environ[k] = "1"
    if deterministic:
        for k in _GTC:
            os.environ.setdefault(k, "0")
        if os.environ.get("MIOPEN_USER_DB_PATH", TUNED_DB) == TUNED_DB:
            det = os.path.join(os.path.expanduser("~"), ".cache", "kca_miopen_deterministic")
            os.makedirs(det, exist_ok=True)
            os.environ["MIOPEN_USER_DB_PATH"] = det
        return
    if os.path.isdir(TUNED_DB) and os.access(TUNED_DB, os.W_OK):
        os.environ.setdefault("MIOPEN_USER_DB_PATH", TUNED_DB)
