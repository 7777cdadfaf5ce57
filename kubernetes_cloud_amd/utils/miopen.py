"""MIOpen convolution-solver policy for the SD UNet / VAE (K15 convolutions).

PyTorch-ROCm asks MIOpen to *find* a solver for every new convolution config.
For the channels-last (NHWC) bf16 convolutions that search also times MIOpen's
reference "naive" direct-convolution solvers, which take seconds per call at
SD-1.5 shapes: a cold UNet training step spent > 3 minutes searching on an
MI355X, and with the naive solvers excluded it takes 5 s (they never win the
search; `MIOPEN_FIND_MODE=FAST` instead picks kernels 4-5x slower). This
matters for the KServe cold start the reference budgets
(online-inference/README.md:14,33) as much as for the finetuner.

``configure()`` runs before the first convolution; explicit environment
settings win.
"""
from __future__ import annotations

import os

_NAIVE = ("MIOPEN_DEBUG_CONV_DIRECT_NAIVE_CONV_FWD", "MIOPEN_DEBUG_CONV_DIRECT_NAIVE_CONV_BWD",
          "MIOPEN_DEBUG_CONV_DIRECT_NAIVE_CONV_WRW")


def configure() -> None:
    for k in _NAIVE:
        os.environ.setdefault(k, "0")
