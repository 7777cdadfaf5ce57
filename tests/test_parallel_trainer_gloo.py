"""3D-parallel trainer on CPU (gloo): TP=2 x PP=2 (GPT-J, untied) and PP=2
(GPT-2, tied embedding) must train to the same weights as a single-process
run over the same micro-batches; sharded checkpoints consolidate back to an
HF directory."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from .helpers import make_model_dir

STEPS, MB, GAS, SEQ = 3, 2, 4, 16


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _args(model_dir, out, tp, pp):
    return ["--model", model_dir, "--tp", str(tp), "--pp", str(pp), "--micro-batch", str(MB), "--gradients",
            str(GAS), "--seq-len", str(SEQ), "--max-steps", str(STEPS), "--lr", "1e-2", "--lr-schedule",
            "constant", "--warmup-ratio", "0", "--output-path", out, "--weight-decay", "0.01"]


def _worker(rank, world, port, model_dir, out, tp, pp):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    from kubernetes_cloud_amd.train.parallel_trainer import main
    main(_args(model_dir, out, tp, pp))
    dist.destroy_process_group()


def _reference(model_dir):
    from kubernetes_cloud_amd.io.hf import load_pretrained
    from kubernetes_cloud_amd.models.config import LMConfig
    from kubernetes_cloud_amd.train.engine import TrainEngine
    m = load_pretrained(model_dir, dtype=torch.float32)
    cfg = LMConfig.from_pretrained(model_dir)
    eng = TrainEngine(m, lr=1e-2, betas=(0.9, 0.95), weight_decay=0.01, max_grad_norm=1.0, grad_accum=GAS)
    g = torch.Generator().manual_seed(42)  # synthetic stream of dp replica 0 (seed + dp_idx)
    for _ in range(STEPS):
        mbs = [torch.randint(0, cfg.vocab_size, (MB, SEQ), generator=g) for _ in range(GAS)]
        for ids in mbs:
            eng.backward(m(ids, labels=ids))
        eng.step(1e-2)
    return m


@pytest.mark.parametrize("preset,tp,pp", [("gpt-j-6b", 2, 2), ("gpt2", 1, 2)])
def test_3d_matches_single_process(preset, tp, pp, tmp_path):
    from kubernetes_cloud_amd.io.hf import load_pretrained
    from kubernetes_cloud_amd.train.parallel_trainer import consolidate
    d = make_model_dir(str(tmp_path / "m"), preset, vocab_size=128, tokenizer=False)
    out = str(tmp_path / "out")
    world = tp * pp
    port = _port()
    ctx = mp.get_context("spawn")
    ps = [ctx.Process(target=_worker, args=(r, world, port, d, out, tp, pp)) for r in range(world)]
    for p in ps:
        p.start()
    for p in ps:
        p.join(timeout=600)
        assert p.exitcode == 0
    ck = os.path.join(out, f"checkpoint-{STEPS}")
    assert len([f for f in os.listdir(ck) if f.startswith("mp_rank_")]) == world
    merged = consolidate(ck, str(tmp_path / "merged"))
    got = load_pretrained(merged, dtype=torch.float32).state_dict()
    ref = _reference(d).state_dict()
    err = max(float((got[k] - ref[k]).abs().max()) for k in ref if not k.endswith("alibi"))
    assert err < 2e-4, err
