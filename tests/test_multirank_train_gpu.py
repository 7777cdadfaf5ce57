"""Multi-rank TRAINING paths rehearsed on the one GPU of the box.

Two (or four) ranks share ``cuda:0`` (``KCA_BENCH_SHARED_GPU=1``:
``parallel.dist.init_distributed`` puts every rank on device 0 with a gloo
default group and installs ``parallel/shared_gpu.py``, which stages device
collectives AND the point-to-point ``batch_isend_irecv`` of the pipeline
stages / Adasum through the host). The 8-GPU driver run is otherwise the first
execution of:

* the NeoX-style 3D trainer (``train/parallel_trainer.py``; the reference's
  gpt-neox/04-finetune-workflow.yaml:199-244) on GPT-J and on the gpt_neox
  architecture itself: TP=2 (column/row backward all-reduces), PP=2 (1F1B P2P
  activations / gradients), DP=2 x TP=2 with ZeRO-1 over the DP group -- each
  against the same trainer at world 1 over the same global batch, within twice
  a measured bf16 noise floor (bf16 both sides);
* the ResNet-50 trainer (``train/resnet.py``, resnet50_pytorch.py:93-125 /
  resnet50_horovod.py:129-140): world 1 on the GPU (channels-last, MIOpen,
  bf16 autocast) and DDP + Adasum at world 2;
* the SD / DreamBooth trainer (``train/sd_finetuner.py``) at world 2.
"""
import os
import subprocess
import sys

import pytest
import torch

from .helpers import make_images, make_model_dir, make_sd_dir

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
STEPS, MB, GAS, SEQ = 3, 2, 4, 64


def _launch(n: int, module: str, argv: list, timeout: int = 400, extra_env: dict | None = None):
    cmd = [sys.executable, "-u", "-m", "kubernetes_cloud_amd.launch", "--num_gpus", str(n), "-m", module] + argv
    env = dict(os.environ, PYTHONPATH=ROOT, KCA_BENCH_SHARED_GPU="1" if n > 1 else "0",
               HSA_ENABLE_IPC_MODE_LEGACY="0", OMP_NUM_THREADS="2", **(extra_env or {}))
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK"):
        env.pop(k, None)
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=timeout)
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-4000:])
    return r


def _neox_args(model_dir, out, tp, pp, zero=0, mb=MB, gas=GAS):
    return ["--model", model_dir, "--tp", str(tp), "--pp", str(pp), "--zero-stage", str(zero),
            "--micro-batch", str(mb), "--gradients", str(gas), "--seq-len", str(SEQ), "--max-steps", str(STEPS),
            "--lr", "1e-3", "--lr-schedule", "constant", "--warmup-ratio", "0", "--output-path", out,
            "--weight-decay", "0.01"]


_ARCH = {"gpt-j-6b": dict(n_embd=256, n_layer=4, n_head=4, rotary_dim=16),
         # gpt_neox: separate ln_2, parallel residual, rotate-half RoPE on 25 % of the 64-wide heads
         "pythia-2.8b": dict(hidden_size=256, num_hidden_layers=4, num_attention_heads=4,
                             intermediate_size=1024)}


def _run_w1(d, out, mb, gas, fp32=False):
    from kubernetes_cloud_amd.io.hf import load_pretrained
    from kubernetes_cloud_amd.train.parallel_trainer import consolidate
    _launch(1, "kubernetes_cloud_amd.train.parallel_trainer",
            _neox_args(d, out, 1, 1, mb=mb, gas=gas) + (["--fp32"] if fp32 else []))
    merged = consolidate(os.path.join(out, f"checkpoint-{STEPS}"), out + "m")
    return load_pretrained(merged, dtype=torch.float32).state_dict(), _metrics(out)


@pytest.fixture(scope="module", params=sorted(_ARCH))
def neox_ref(request, tmp_path_factory):
    """World-1 references on the GPU, per architecture: the step's global batch at micro-batch MB
    (for the TP / PP layouts) and at 2 x MB (what a DP=2 layout of micro-batch MB consumes per step),
    each in bf16 and in fp32 (the exact result the bf16 runs approximate), plus a reduction-order run
    -- the same global batch as MB x GAS split into 2 x GAS micro-batches of MB / 2."""
    from kubernetes_cloud_amd.io.hf import load_pretrained
    arch = request.param
    tmp = tmp_path_factory.mktemp(arch.replace(".", "_"))
    d = make_model_dir(str(tmp / "m"), arch, vocab_size=256, tokenizer=False, **_ARCH[arch])
    init = load_pretrained(d, dtype=torch.float32).state_dict()
    ref = _run_w1(d, str(tmp / "w1"), MB, GAS)
    alt = _run_w1(d, str(tmp / "w1alt"), MB // 2, 2 * GAS)
    ref2 = _run_w1(d, str(tmp / "w1x2"), 2 * MB, GAS)
    ref32 = _run_w1(d, str(tmp / "w1f32"), MB, GAS, fp32=True)
    ref2_32 = _run_w1(d, str(tmp / "w1x2f32"), 2 * MB, GAS, fp32=True)
    return arch, d, tmp, init, ref, alt, ref2, ref32, ref2_32


def _metrics(out):
    import json
    with open(os.path.join(out, "logs", "parallel-trainer.metrics.jsonl")) as f:
        rows = [json.loads(ln) for ln in f if ln.strip()]
    return [r["train/loss"] for r in rows], [r["train/grad_norm"] for r in rows]


def _rel(got, ref, init):
    """Per tensor ||got - ref|| / ||ref - init|| (the size of the difference against the size of the
    update itself)."""
    out = {}
    for k in ref:
        if k.endswith("alibi"):
            continue
        dn = (ref[k] - init[k]).norm()
        if dn > 0:
            out[k] = float((got[k] - ref[k]).norm() / dn)
    return out


@pytest.mark.parametrize("tp,pp,dp,zero", [(2, 1, 1, 0), (1, 2, 1, 0), (2, 1, 2, 1)])
def test_neox_3d_trainer_on_gpu_matches_world1(neox_ref, tp, pp, dp, zero):
    """TP=2, PP=2 and DP=2 x TP=2 (ZeRO-1) against world 1 over the same global batch: loss curve,
    gradient norm (the clip's global norm: a wrong all-reduce scale moves it by the scale factor) and
    every parameter after 3 Adam steps. The bf16 layouts are compared with the fp32 world-1 run (the
    exact result): each may be at most twice as far from it as the bf16 world-1 run is -- the measured
    bf16 noise floor. (A TP layout rounds each row-parallel partial output to bf16 before its
    all-reduce, as Megatron / GPT-NeoX do; that is a rounding the world-1 run does not make, so the
    floor is the distance to the exact result, not a reduction-order spread.)"""
    from kubernetes_cloud_amd.io.hf import load_pretrained
    from kubernetes_cloud_amd.train.parallel_trainer import consolidate
    arch, d, tmp, init, ref, alt, ref2, ref32, ref2_32 = neox_ref
    tag = f"tp{tp}pp{pp}dp{dp}"
    out = str(tmp / tag)
    _launch(tp * pp * dp, "kubernetes_cloud_amd.train.parallel_trainer", _neox_args(d, out, tp, pp, zero))
    ck = os.path.join(out, f"checkpoint-{STEPS}")
    assert len([f for f in os.listdir(ck) if f.startswith("mp_rank_")]) == tp * pp
    got = load_pretrained(consolidate(ck, str(tmp / (tag + "m"))), dtype=torch.float32).state_dict()
    (sd_r, (l_r, g_r)), (sd_t, (l_t, g_t)) = (ref2, ref2_32) if dp > 1 else (ref, ref32)
    l_g, g_g = _metrics(out)
    assert len(l_g) == len(l_r) == len(l_t) == STEPS
    med = lambda d_: sorted(d_.values())[len(d_) // 2]  # noqa: E731
    floor = _rel(sd_r, sd_t, init)  # bf16 world 1 against the exact result
    rel = _rel(got, sd_t, init)
    n_med, n_max, r_med, r_max = med(floor), max(floor.values()), med(rel), max(rel.values())
    loss_tol = 2 * max(abs(a - b) for a, b in zip(l_r, l_t)) + 1e-3
    gn_tol = 2 * max(abs(a - b) for a, b in zip(g_r, g_t)) + 1e-3 * max(g_t)
    report = dict(arch=arch, floor=(n_med, n_max), got=(r_med, r_max), loss=(l_t, l_r, l_g), gn=(g_t, g_r, g_g),
                  worst=sorted(rel.items(), key=lambda kv: -kv[1])[:4])
    assert all(abs(a - b) <= loss_tol for a, b in zip(l_t, l_g)), report
    assert all(abs(a - b) <= gn_tol for a, b in zip(g_t, g_g)), report
    assert r_med <= 2 * n_med + 1e-3 and r_max <= 2 * n_max + 1e-3, report
    # the bounds discriminate: a gradient scaled by 2 (sum instead of mean over 2 replicas) moves the
    # logged norm past gn_tol, and the update of a different global batch (a replica that never
    # reduced: the MB-row reference against the 2 x MB one) lies outside the parameter bound
    assert gn_tol < min(g_t), report
    other = _rel(ref2[0] if dp == 1 else ref[0], sd_t, init)
    assert med(other) > 2 * n_med + 1e-3, (report, other)
    # (the reduction-order run stays inside the same bound: the floor is not an over-estimate)
    assert med(_rel(alt[0], ref32[0], init)) <= 2 * med(_rel(ref[0], ref32[0], init)) + 1e-3


def test_resnet_trainer_gpu_world1_and_ddp_adasum_world2(tmp_path):
    common = ["--synthetic", "16", "--batch-size", "4", "--epochs", "1", "--max-steps", "3",
              "--train-crop-size", "64", "--val-crop-size", "64", "--workers", "0", "--num-classes", "10",
              "--use-mixed-precision"]
    r1 = _launch(1, "kubernetes_cloud_amd.train.resnet", common + ["--log-dir", str(tmp_path / "l1")])
    assert "Test Epoch: 1" in r1.stdout
    r2 = _launch(2, "kubernetes_cloud_amd.train.resnet", common + ["--use-adasum", "--log-dir",
                                                                  str(tmp_path / "l2")])
    assert "Test Epoch: 1" in r2.stdout


def _sd_run(d, data, out, world, batch, extra_env=None):
    import glob
    import json

    from safetensors.torch import load_file
    argv = ["--model", d, "--run_name", "w", "--dataset", data, "--resolution", "32", "--batch_size", str(batch),
            "--epochs", "1", "--output_path", out, "--image_log_steps", "0", "--save_steps", "0", "--ucg", "0",
            "--shuffle", "False", "--lr", "1e-4"]
    _launch(world, "kubernetes_cloud_amd.train.sd_finetuner", argv, extra_env=extra_env)
    sd = load_file(glob.glob(os.path.join(out, "unet", "*.safetensors"))[0])
    with open(os.path.join(out, "logs", "w.metrics.jsonl")) as f:
        rows = [json.loads(ln) for ln in f if ln.strip()]
    return {k: v.float() for k, v in sd.items()}, [r["train/loss"] for r in rows], [r["train/grad_norm"] for r in rows]


def test_sd_trainer_world2_matches_world1_on_gpu(tmp_path):
    """The SD trainer (PAR-7: accelerate-style DDP, sd-finetuner/finetuner.py:532-534) at world 2 x batch 1
    against world 1 x batch 2 over the same samples: one interleaving sampler for every world size,
    timesteps and noise drawn per GLOBAL sample. Loss (the all-reduced step loss), the clip's global
    gradient norm and the UNet after 2 steps agree within twice the measured bf16 noise floor (the same
    world-1 run with unpadded training attention heads: same math, other kernels)."""
    from safetensors.torch import load_file
    import glob
    d = make_sd_dir(str(tmp_path / "sd"))
    init = {k: v.float() for k, v in load_file(glob.glob(os.path.join(d, "unet", "*.safetensors"))[0]).items()}
    data = make_images(str(tmp_path / "data"), 4)
    ref, l_r, g_r = _sd_run(d, data, str(tmp_path / "w1"), 1, 2)
    alt, l_a, g_a = _sd_run(d, data, str(tmp_path / "w1alt"), 1, 2, {"KCA_SD_PAD_HEADS_TRAIN": "0"})
    got, l_g, g_g = _sd_run(d, data, str(tmp_path / "w2"), 2, 1)
    assert len(l_r) == len(l_g) == 2
    noise, rel = _rel(alt, ref, init), _rel(got, ref, init)
    n_med, n_max = sorted(noise.values())[len(noise) // 2], max(noise.values())
    r_med, r_max = sorted(rel.values())[len(rel) // 2], max(rel.values())
    loss_tol = 2 * max(abs(a - b) for a, b in zip(l_a, l_r)) + 1e-4 * max(l_r)
    gn_tol = 2 * max(abs(a - b) for a, b in zip(g_a, g_r)) + 1e-3 * max(g_r)
    report = dict(noise=(n_med, n_max), got=(r_med, r_max), loss=(l_r, l_g, l_a), gn=(g_r, g_g, g_a))
    assert all(abs(a - b) <= loss_tol for a, b in zip(l_r, l_g)), report
    assert all(abs(a - b) <= gn_tol for a, b in zip(g_r, g_g)), report
    assert r_med <= 2 * n_med + 1e-3 and r_max <= 2 * n_max + 1e-3, report
    assert gn_tol < min(g_r), report  # a gradient scaled by the world size would fail the norm bound


def test_sd_trainer_world2_on_gpu(tmp_path):
    d = make_sd_dir(str(tmp_path / "sd"))
    data = make_images(str(tmp_path / "data"), 4)
    argv = ["--model", d, "--run_name", "w2", "--dataset", data, "--resolution", "32", "--batch_size", "1",
            "--epochs", "1", "--output_path", str(tmp_path / "o"), "--image_log_steps", "0", "--save_steps", "0"]
    r = _launch(2, "kubernetes_cloud_amd.train.sd_finetuner", argv)
    outs = [os.path.join(dp, f) for dp, _, fs in os.walk(str(tmp_path / "o")) for f in fs]
    assert any("unet" in p for p in outs), (outs[:20], r.stderr[-2000:])
