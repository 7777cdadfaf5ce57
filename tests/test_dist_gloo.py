"""Multi-process CPU tests (gloo, world_size 2): the bucketed ZeRO engine must
produce the same parameters as a single-process run over the same global
batch, and the launcher must run the finetuner CLI across ranks."""
import os
import socket
import subprocess
import sys

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _model(seed=0):
    from kubernetes_cloud_amd.models.causal_lm import build_model
    from kubernetes_cloud_amd.models.config import PRESETS_HF, LMConfig
    cfg = dict(PRESETS_HF["gpt-j-6b"])
    cfg.update(n_embd=64, n_layer=2, n_head=4, rotary_dim=8, vocab_size=256)
    return build_model(LMConfig.from_hf(cfg), dtype=torch.float32, seed=seed)


def _batches(world, gas, bs=2, seq=16, steps=3):
    g = torch.Generator().manual_seed(123)
    return [[torch.randint(0, 256, (bs * world, seq), generator=g) for _ in range(gas)] for _ in range(steps)]


def _worker(rank, world, port, stage, bucket, out_path):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from kubernetes_cloud_amd.train.engine import TrainEngine
    m = _model()
    eng = TrainEngine(m, lr=1e-2, weight_decay=0.01, zero_stage=stage, grad_accum=2, bucket_elems=bucket)
    for step in _batches(world, 2):
        mbs = [b[rank * 2:(rank + 1) * 2] for b in step]
        eng.train_batch(mbs, lambda ids: m(ids, labels=ids))
    if rank == 0:
        torch.save({k: v.detach().clone() for k, v in m.state_dict().items()}, out_path)
    dist.barrier()
    dist.destroy_process_group()


def _reference():
    from kubernetes_cloud_amd.train.engine import TrainEngine
    m = _model()
    eng = TrainEngine(m, lr=1e-2, weight_decay=0.01, zero_stage=0, grad_accum=2)
    for step in _batches(2, 2):
        # global batch of 4 per micro-step, same mean as 2 ranks x 2
        def lf(ids):
            return 0.5 * (m(ids[:2], labels=ids[:2]) + m(ids[2:], labels=ids[2:]))
        eng.train_batch(step, lf)
    return {k: v.detach().clone() for k, v in m.state_dict().items()}


@pytest.mark.parametrize("stage,bucket", [(0, 10_000), (1, 10_000), (2, 3_000)])
def test_engine_dp_matches_single_process(stage, bucket, tmp_path):
    ctx = mp.get_context("spawn")
    port = _port()
    out = str(tmp_path / "sd.pt")
    ps = [ctx.Process(target=_worker, args=(r, 2, port, stage, bucket, out)) for r in range(2)]
    for p in ps:
        p.start()
    for p in ps:
        p.join(timeout=300)
        assert p.exitcode == 0
    got = torch.load(out, weights_only=True)
    ref = _reference()
    for k in ref:
        assert torch.allclose(got[k], ref[k], atol=2e-5, rtol=1e-4), k


def test_launcher_runs_finetuner_two_ranks(tmp_path):
    from .helpers import make_model_dir, make_tokens
    model = make_model_dir(str(tmp_path / "m"))
    data = make_tokens(str(tmp_path / "d.tokens"), n_ctx=16, ctx=16)
    cmd = [sys.executable, "-m", "kubernetes_cloud_amd.launch", "--num_gpus", "2", "-m",
           "kubernetes_cloud_amd.train.finetuner", "--run-name", "dd", "--model", model, "--dataset", data,
           "--context-size", "16", "--bs", "2", "--gradients", "1", "--output-path", str(tmp_path / "o"),
           "--logs", str(tmp_path / "l"), "--save-steps", "2", "--max-steps", "2", "--zero-stage", "2"]
    env = dict(os.environ, PYTHONPATH=ROOT, CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="")
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=400)
    assert r.returncode == 0, r.stderr[-3000:]
    rd = tmp_path / "o" / "results-dd"
    assert (rd / "checkpoint-2" / "optimizer" / "rank-00001.safetensors").exists()
    assert (rd / "final" / ".ready.txt").exists()
