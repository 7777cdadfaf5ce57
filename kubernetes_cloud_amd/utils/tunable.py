"""PyTorch TunableOp (hipBLASLt / rocBLAS solution search per GEMM shape) with
results files shipped under ``tuning/``.

hipBLASLt's default heuristic picks poorly for some of the framework's GEMMs:
the SD UNet's weight-gradient GEMMs (320 x 320 outputs reduced over 65k
tokens) land on a 64x64 macro tile without split-K -- 25 workgroups on a
256-CU chip. TunableOp times the candidate solutions once on an MI355X and
records the winner; ``configure(..., "use")`` replays those choices with no
search. Files: ``tuning/tunableop_results.csv`` (GPT-J-6B training step) and
``tuning/tunableop_sd.csv`` (SD-1.5 DreamBooth step + txt2img UNet),
``tuning/tunableop_decode.csv`` (serving decode / prefill GEMMs, loaded by
``engine.runner.ModelRunner`` on the GPU).
"""
from __future__ import annotations

import os

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
GPTJ_FILE = os.path.join(ROOT, "tuning", "tunableop_results.csv")
SD_FILE = os.path.join(ROOT, "tuning", "tunableop_sd.csv")
# serving: the decode-step GEMMs at batch buckets 2..64 (M = batch, K/N = model dims), where
# hipBLASLt's default heuristic picks long split-free K loops (GPT-J fc_out at M=64: 0.9 TB/s)
DECODE_FILE = os.path.join(ROOT, "tuning", "tunableop_decode.csv")


def configure(path: str, mode: str = "auto", max_tuning_ms: int = 40) -> str:
    """mode: 'use' replays ``path``; 'tune' searches unseen shapes and writes
    ``path`` at exit; 'auto' = 'use' when ``path`` exists else 'off'.
    Returns the mode applied."""
    if mode == "auto":
        mode = "use" if os.path.exists(path) else "off"
    if mode == "off":
        return mode
    import torch.cuda.tunable as tunable

    os.makedirs(os.path.dirname(path), exist_ok=True)
    tunable.enable(True)
    tunable.set_filename(path, insert_device_ordinal=False)
    tunable.tuning_enable(mode == "tune")
    if mode == "tune":
        tunable.set_max_tuning_duration(max_tuning_ms)
    if os.path.exists(path):
        tunable.read_file(path)
    return mode


def add_results(path: str) -> bool:
    """Merge another results file into the live table (e.g. the SD file after
    the GPT-J one in bench.py)."""
    if not os.path.exists(path):
        return False
    import torch.cuda.tunable as tunable

    return bool(tunable.read_file(path))


def ensure(path: str) -> None:
    """Make ``path``'s results active: merged into the live table when TunableOp
    is already on (e.g. the GPT-J file in bench.py), else enabled in 'use' mode
    when the file exists. Unlisted shapes keep hipBLASLt's default heuristic.
    ``KCA_TUNABLEOP=off`` disables (the benches' ``--tunableop off`` sets it)."""
    if os.environ.get("KCA_TUNABLEOP", "auto") == "off":
        return
    import torch.cuda.tunable as tt

    if tt.is_enabled():
        add_results(path)
    else:
        configure(path, "auto")
