"""ResNet-50 DDP (train/resnet.py, resnet50_pytorch.py:93-125) at world 2 against a world-1 reference.

Each DDP rank normalises its own half of the global batch (per-replica BatchNorm, as the reference's
DDP job does), so the exact world-1 counterpart is the global batch through the same model with the
BatchNorm statistics taken per half ("ghost" BatchNorm): the two halves forward separately, the loss is
their mean, and SGD runs at the world-2 learning rate (lr x world, resnet50_horovod.py:121-123). The
parameter UPDATES (final - initial) after the trainer's steps must agree within 2x a measured fp32
noise floor (the same reference with the two halves' gradients accumulated by two backward passes
instead of one: another summation order), and the check must reject a reference whose gradient is
scaled as a wrong all-reduce would scale it. CPU / gloo; the trainer's ranks and the reference both
run 2 threads (oneDNN picks other convolution algorithms at other thread counts, and BatchNorm over
4-sample halves amplifies that into percent-level differences within a few steps).
"""
import os
import subprocess
import sys

import torch
import torch.nn.functional as F

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
N, BATCH, CROP, CLASSES, STEPS, LR, SEED = 32, 4, 64, 10, 3, 0.001, 1


def _run_ddp(tmp_path):
    out = tmp_path / "model"
    cmd = [sys.executable, "-m", "kubernetes_cloud_amd.launch", "--num_gpus", "2", "-m",
           "kubernetes_cloud_amd.train.resnet", "--no-cuda", "--synthetic", str(N), "--batch-size", str(BATCH),
           "--epochs", "1", "--max-steps", str(STEPS), "--train-crop-size", str(CROP), "--val-crop-size",
           str(CROP), "--workers", "0", "--num-classes", str(CLASSES), "--lr", str(LR), "--seed", str(SEED),
           "--log-dir", str(tmp_path / "logs"), "--model-dir", str(out), "--log-interval", "1"]
    env = dict(os.environ, PYTHONPATH=ROOT, CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="", OMP_NUM_THREADS="2")
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK"):
        env.pop(k, None)
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-3000:])
    return torch.load(out / "resnet50_imagenet.pt", weights_only=True)


def _reference(world=2, grad_scale=1.0, split_backward=False, threads=2):
    """World 1, global batch = the two ranks' batches, BatchNorm per half, mean of the half losses.
    Returns (final, initial) state dicts."""
    from torch.utils.data import DistributedSampler
    prev = torch.get_num_threads()
    torch.set_num_threads(threads)
    try:
        return _reference_run(world, grad_scale, split_backward, DistributedSampler)
    finally:
        torch.set_num_threads(prev)


def _reference_run(world, grad_scale, split_backward, DistributedSampler):
    from kubernetes_cloud_amd.models.resnet import resnet50
    from kubernetes_cloud_amd.train.resnet import Synthetic
    torch.manual_seed(SEED)
    ds = Synthetic(N, CROP, CLASSES)
    model = resnet50(CLASSES)
    model.train()
    init = {k: v.detach().clone() for k, v in model.state_dict().items()}
    opt = torch.optim.SGD(model.parameters(), lr=LR * world, momentum=0.9)
    orders = []
    for r in range(world):
        s = DistributedSampler(ds, num_replicas=world, rank=r, shuffle=True, seed=SEED)
        s.set_epoch(1)
        orders.append(list(s))
    for step in range(STEPS):
        opt.zero_grad(set_to_none=True)
        losses = []
        for r in range(world):
            idx = orders[r][step * BATCH:(step + 1) * BATCH]
            x = torch.stack([ds[i][0] for i in idx])
            y = torch.tensor([ds[i][1] for i in idx])
            loss = F.cross_entropy(model(x).float(), y)
            if split_backward:
                (loss * (grad_scale / world)).backward()
            else:
                losses.append(loss)
        if not split_backward:
            (sum(losses) / world * grad_scale).backward()
        opt.step()
    return {k: v.detach().clone() for k, v in model.state_dict().items()}, init


def _upd_rel(a, b, init):
    """Relative distance of the parameter updates (a - init vs b - init) over all trainable tensors."""
    num = den = 0.0
    for k, v in b.items():
        if not v.is_floating_point() or "running" in k:  # running stats: rank 0's half only under DDP
            continue
        db = v.float() - init[k].float()
        num += float((a[k].float() - v.float()).pow(2).sum())
        den += float(db.pow(2).sum())
    return (num / max(den, 1e-30)) ** 0.5


def test_resnet_ddp_world2_matches_ghost_bn_world1(tmp_path):
    ddp = _run_ddp(tmp_path)
    ref, init = _reference()
    floor = _upd_rel(_reference(split_backward=True)[0], ref, init)  # fp32 noise: another summation order
    tol = max(2 * floor, 1e-6)
    err = _upd_rel(ddp, ref, init)
    assert err <= tol, (err, floor)
    # a wrong all-reduce scale (the sum instead of the mean: x2) must not pass the same check
    wrong = _upd_rel(ddp, _reference(grad_scale=2.0)[0], init)
    assert wrong > 10 * tol, (wrong, tol)
