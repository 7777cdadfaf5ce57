"""Multi-rank rehearsal on the one GPU of the box.

The driver's 8-GPU scaling bench is otherwise the first execution of the N>1
paths. Here two ranks share ``cuda:0`` (``parallel/shared_gpu.py``: gloo
default group, device collectives staged through the host; the custom xGMI
all-reduce / all-gather map each other's IPC buffers exactly as on two
devices):

* ``bench.py --gpus 2`` end to end with a shrunk GPT-J (ZeRO-1 over 2 ranks)
  and BLOOM-176B TP=2 cut to 2 layers (``run_tp_decode``: ``load_tp_model``
  random-init, ``register(None)`` custom all-reduce, decode graphs holding the
  xGMI all-reduce + all-gather and no RCCL call, gloo control plane);
* ``TrainEngine`` ZeRO stages 1/2/3 at world 2 on the GPU against stage 0 at
  world 2 and against a one-process run over the same global batch.
"""
import json
import os
import socket
import subprocess
import sys

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_bench_two_ranks_shared_gpu():
    cmd = [sys.executable, "-u", os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "2", "--warmup", "1",
           "--layers", "2", "--hidden", "1024", "--heads", "4", "--seq", "512", "--micro-batch", "2", "--gas", "2",
           "--sd", "0", "--bloom-layers", "2", "--bloom-batches", "1,4", "--bloom-timeout", "240",
           "--tunableop", "off"]
    env = dict(os.environ, KCA_BENCH_SHARED_GPU="1", HSA_ENABLE_IPC_MODE_LEGACY="0")
    env.pop("WORLD_SIZE", None)
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=400)
    sys.stderr.write(r.stderr[-4000:])
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    rec = json.loads(lines[0])
    assert rec["n_gpus"] == 2
    assert rec["config"]["parallelism"] == "dp2-zero1"
    assert rec["config"]["rehearsal"]["shared_gpu"] is True
    assert rec["value"] > 0
    bloom = rec["bloom_tp"]
    assert isinstance(bloom, list) and len(bloom) == 2, bloom
    for b in bloom:
        assert "error" not in b, b
        assert b["tp"] == 2 and b["custom_allreduce"] is True, b
        assert b["decode_ms_per_token"] > 0


# ------------------------------------------------------------ ZeRO parity
def _model(dev, seed=0):
    from kubernetes_cloud_amd.models.causal_lm import build_model
    from kubernetes_cloud_amd.models.config import PRESETS_HF, LMConfig
    cfg = dict(PRESETS_HF["gpt-j-6b"])
    cfg.update(n_embd=256, n_layer=2, n_head=4, rotary_dim=16, vocab_size=512)
    return build_model(LMConfig.from_hf(cfg), device=dev, dtype=torch.bfloat16, seed=seed)


def _batches(gas=2, bs=2, seq=64, steps=3):
    """Global batch of 2 ranks x ``bs`` rows per micro-step."""
    g = torch.Generator().manual_seed(123)
    return [[torch.randint(0, 512, (bs * 2, seq), generator=g) for _ in range(gas)] for _ in range(steps)]


def _train(stage, rank, world, dev):
    from kubernetes_cloud_amd.train.engine import TrainEngine
    m = _model(dev)
    m.train()
    eng = TrainEngine(m, lr=1e-2, weight_decay=0.01, zero_stage=stage, grad_accum=2, bucket_elems=50_000)
    mem = eng.memory_report()
    for step in _batches():
        if world > 1:
            mbs = [b[rank * 2:(rank + 1) * 2].to(dev) for b in step]
            eng.train_batch(mbs, lambda ids: m(ids, labels=ids))
        else:
            def lf(ids):
                return sum(m(ids[2 * r:2 * r + 2], labels=ids[2 * r:2 * r + 2]) for r in range(2)) / 2
            eng.train_batch([b.to(dev) for b in step], lf)
    torch.cuda.synchronize()
    if stage == 3 and world > 1:
        assert all(p.numel() == 0 for p in m.parameters()), "ZeRO-3 params not released"
    with eng.gathered():
        sd = {k: v.detach().float().cpu().clone() for k, v in m.state_dict().items()}
    eng.remove_hooks()
    return sd, mem


def _zero_worker(rank, world, port, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), HSA_ENABLE_IPC_MODE_LEGACY="0")
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from kubernetes_cloud_amd.parallel import shared_gpu
    shared_gpu.install()
    dev = torch.device("cuda", 0)
    res = {}
    for stage in (0, 1, 2, 3):
        res[stage] = _train(stage, rank, world, dev)
        dist.barrier()
    if rank == 0:
        torch.save({s: {"sd": v[0], "mem": v[1]} for s, v in res.items()}, out)
    dist.barrier()
    dist.destroy_process_group()


def _close(a, b):
    """bf16 AdamW after 3 steps: implementations that differ only in fp32
    reduction order agree on all but a few elements; a wrong or missing
    gradient reduction moves a large fraction of them the other way."""
    d = (a - b).abs()
    # one bf16 ulp is 7.8e-3 at 1.0 (LayerNorm weights): the bound scales with |b|; a wrong
    # update moves a ~0.02 weight by 2 x lr = 2e-2
    return float(d.mean()), float((d > 4e-3 + 1e-2 * b.abs()).float().mean())


def test_zero_stages_world2_on_gpu_match(tmp_path):
    out = str(tmp_path / "zero.pt")
    ctx = mp.get_context("spawn")
    port = _port()
    ps = [ctx.Process(target=_zero_worker, args=(r, 2, port, out)) for r in range(2)]
    for p in ps:
        p.start()
    for p in ps:
        p.join(timeout=300)
        assert p.exitcode == 0
    res = torch.load(out, weights_only=True)
    single, _ = _train(0, 0, 1, torch.device("cuda", 0))
    base = res[0]["sd"]
    for k in base:
        mean, frac = _close(base[k], single[k])
        assert mean < 1e-3 and frac < 0.02, ("stage0 world2 vs world1", k, mean, frac)
    for stage in (1, 2, 3):
        got = res[stage]["sd"]
        for k in base:
            mean, frac = _close(got[k], base[k])
            assert mean < 1e-3 and frac < 0.02, (stage, k, mean, frac)
    m1, m2, m3 = (res[s]["mem"] for s in (1, 2, 3))
    assert (m1["zero_stage"], m2["zero_stage"], m3["zero_stage"]) == (1, 2, 3)
    assert m2["grads_fp32"] < m1["grads_fp32"]
    assert m3["params_bf16"] < m2["params_bf16"]
