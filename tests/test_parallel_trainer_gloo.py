"""3D-parallel trainer on CPU (gloo): TP=2 x PP=2 (GPT-J, untied), PP=2
(GPT-2, tied embedding) and DP=2 x TP=2 x PP=2 with ZeRO-1 over the DP group
(the reference's NeoX layout, gpt-neox/04-finetune-workflow.yaml:199-244) must
train to the same weights as a single-process run over the same global
micro-batches; sharded checkpoints consolidate back to an HF directory."""
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


def _args(model_dir, out, tp, pp, zero=1):
    return ["--model", model_dir, "--tp", str(tp), "--pp", str(pp), "--zero-stage", str(zero),
            "--micro-batch", str(MB), "--gradients",
            str(GAS), "--seq-len", str(SEQ), "--max-steps", str(STEPS), "--lr", "1e-2", "--lr-schedule",
            "constant", "--warmup-ratio", "0", "--output-path", out, "--weight-decay", "0.01"]


def _worker(rank, world, port, model_dir, out, tp, pp, zero):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    torch.set_num_threads(1)
    from kubernetes_cloud_amd.train.parallel_trainer import main
    main(_args(model_dir, out, tp, pp, zero))
    dist.destroy_process_group()


def _reference(model_dir, dp=1):
    from kubernetes_cloud_amd.io.hf import load_pretrained
    from kubernetes_cloud_amd.models.config import LMConfig
    from kubernetes_cloud_amd.train.engine import TrainEngine
    m = load_pretrained(model_dir, dtype=torch.float32)
    cfg = LMConfig.from_pretrained(model_dir)
    eng = TrainEngine(m, lr=1e-2, betas=(0.9, 0.95), weight_decay=0.01, max_grad_norm=1.0, grad_accum=GAS)
    g = torch.Generator().manual_seed(42)  # the step's global batch; replica d takes its contiguous share
    for _ in range(STEPS):
        rows = torch.randint(0, cfg.vocab_size, (dp * MB * GAS, SEQ), generator=g)
        mbs = [[rows[d * MB * GAS + k * MB:d * MB * GAS + (k + 1) * MB] for k in range(GAS)] for d in range(dp)]
        for k in range(GAS):
            eng.backward(sum(m(mbs[d][k], labels=mbs[d][k]) for d in range(dp)) / dp)
        eng.step(1e-2)
    return m


@pytest.mark.parametrize("preset,tp,pp,dp,zero", [("gpt-j-6b", 2, 2, 1, 0), ("gpt2", 1, 2, 1, 0),
                                                  ("gpt-j-6b", 2, 2, 2, 1), ("gpt2", 1, 2, 2, 1),
                                                  ("gpt-j-6b", 2, 1, 2, 2)])
def test_3d_matches_single_process(preset, tp, pp, dp, zero, tmp_path):
    from kubernetes_cloud_amd.io.hf import load_pretrained
    from kubernetes_cloud_amd.train.parallel_trainer import consolidate
    d = make_model_dir(str(tmp_path / "m"), preset, vocab_size=128, tokenizer=False)
    out = str(tmp_path / "out")
    world = tp * pp * dp
    port = _port()
    ctx = mp.get_context("spawn")
    ps = [ctx.Process(target=_worker, args=(r, world, port, d, out, tp, pp, zero)) for r in range(world)]
    for p in ps:
        p.start()
    for p in ps:
        p.join(timeout=600)
        assert p.exitcode == 0
    ck = os.path.join(out, f"checkpoint-{STEPS}")
    assert len([f for f in os.listdir(ck) if f.startswith("mp_rank_")]) == tp * pp
    merged = consolidate(ck, str(tmp_path / "merged"))
    got = load_pretrained(merged, dtype=torch.float32).state_dict()
    ref = _reference(d, dp).state_dict()
    # fp32 both sides; Adam moves an element whose gradient is at the reduction-order noise level by up
    # to ~lr either way, so the bound is a few percent of one step (lr 1e-2), not machine epsilon
    err = max(float((got[k] - ref[k]).abs().max()) for k in ref if not k.endswith("alibi"))
    assert err < 5e-4, err
