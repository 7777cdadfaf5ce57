"""Diagnostic: world-1 GPT-J-tiny training with and without batched small-gradient accumulation
(KCA_MULTI_ACCUM) -- identical fp32 arithmetic, so the parameters must match bit for bit."""
import os
import subprocess
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def run(out):
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from test_multirank_gpu import _train
    sd, _ = _train(0, 0, 1, torch.device("cuda", 0))
    torch.save(sd, out)


if __name__ == "__main__":
    if len(sys.argv) > 1:
        run(sys.argv[1])
        sys.exit(0)
    outs = {}
    arms = {"0": {"KCA_MULTI_ACCUM": "0"}, "1": {"KCA_MULTI_ACCUM": "1"},
            "1t": {"KCA_MULTI_ACCUM": "1", "KCA_FLUSH_TORCH": "1"}, "0b": {"KCA_MULTI_ACCUM": "0"}}
    for v, env in arms.items():
        o = f"/tmp/accdbg_{v}.pt"
        subprocess.run([sys.executable, __file__, o], check=True, env=dict(os.environ, **env))
        outs[v] = torch.load(o, weights_only=True)
    for k in outs["0"]:
        print(f"{k:28s} " + " ".join(f"{v}:{(outs['0'][k] - outs[v][k]).abs().max().item():.2e}" for v in arms))
