"""ResNet-50 ImageNet data-parallel trainer (T13).

CLI = the union of resnet50_pytorch.py:28-70 and resnet50_horovod.py:18-62
(``--batch-size`` 64, ``--epochs`` 10, ``--lr`` 0.01 (x world size),
``--momentum`` .9, ``--no-cuda``, ``--seed``, ``--log-interval``, ``--log-dir``,
``--data-dir`` (train/ + val/ ImageFolder), ``--model-dir``, ``--interpolation``,
``--val-resize-size`` 256, ``--val-crop-size``/``--train-crop-size`` 224,
``-j/--workers``, ``--wandb-project``/``--wandb-run``, ``--backend``; Horovod's
``--fp16-allreduce``, ``--use-mixed-precision``, ``--gradient-predivide-factor``,
``--use-adasum``: Horovod's Adasum combination (resnet50_horovod.py:115-139;
``adasum_hook``, recursive doubling with per-tensor coefficients). On GPUs it is
Horovod's hierarchical form: gradients are AVERAGED inside the node and
combined with Adasum across nodes (one cross-node group per local rank), with
the LR scaled by the local size (resnet50_horovod.py:121-123); on CPU it is
flat Adasum over all ranks at LR x 1 ("Adasum doesn't need scaling up learning
rate", :115-116).

MI355X choices: DDP over RCCL with 100 MB buckets (fewer, larger ring
all-reduces over the point-to-point xGMI links), gradient all-reduce
overlapped with backward, channels_last + bf16 autocast (no loss scaler
needed), ``--fp16-allreduce`` = bf16-compressed gradient buckets, rank-0
checkpoint ``resnet50_imagenet.pt`` (resnet50_pytorch.py:143-145), top-1/top-5
accuracy (util.py:150-166). ``--synthetic N`` trains on random tensors (bench /
tests; no dataset offline).
"""
from __future__ import annotations

import argparse
import csv
import os
import shutil
import time
from pathlib import Path

import torch
import torch.distributed as dist
import torch.nn as nn
import torch.nn.functional as F

MEAN = (0.485, 0.456, 0.406)
STD = (0.229, 0.224, 0.225)
IMG_EXT = (".jpg", ".jpeg", ".png", ".bmp", ".JPEG")


def build_parser():
    p = argparse.ArgumentParser(description="ResNet-50 ImageNet (MI355X DDP)")
    p.add_argument("--batch-size", type=int, default=64)
    p.add_argument("--epochs", type=int, default=10)
    p.add_argument("--lr", type=float, default=0.01)
    p.add_argument("--momentum", type=float, default=0.9)
    p.add_argument("--no-cuda", action="store_true", default=False)
    p.add_argument("--seed", type=int, default=1)
    p.add_argument("--log-interval", type=int, default=10)
    p.add_argument("--log-dir", type=Path, default=Path("./logs"))
    p.add_argument("--data-dir", type=Path, default=Path("./data"))
    p.add_argument("--model-dir", type=Path, default=None)
    p.add_argument("--interpolation", default="bilinear", type=str)
    p.add_argument("--val-resize-size", default=256, type=int)
    p.add_argument("--val-crop-size", default=224, type=int)
    p.add_argument("--train-crop-size", default=224, type=int)
    p.add_argument("-j", "--workers", default=16, type=int)
    p.add_argument("--wandb-project", type=str, default=None)
    p.add_argument("--wandb-run", type=str, default=None)
    p.add_argument("--backend", type=str, default=None, help="nccl (RCCL) on GPUs, gloo on CPU")
    p.add_argument("--fp16-allreduce", action="store_true", default=False)
    p.add_argument("--use-mixed-precision", action="store_true", default=False)
    p.add_argument("--use-adasum", action="store_true", default=False)
    p.add_argument("--gradient-predivide-factor", type=float, default=1.0)
    p.add_argument("--bucket-mb", type=int, default=100)
    p.add_argument("--synthetic", type=int, default=0, help="N synthetic samples per epoch instead of data-dir")
    p.add_argument("--num-classes", type=int, default=1000)
    p.add_argument("--max-steps", type=int, default=0)
    p.add_argument("--prepare-val", action="store_true", help="sort val images into class folders and exit")
    p.add_argument("--val-labels", type=Path, default=None)
    p.add_argument("--local_rank", "--local-rank", type=int, default=-1)
    return p


# ------------------------------------------------------------------ data
class ImageFolder(torch.utils.data.Dataset):
    def __init__(self, root: Path, train: bool, args):
        root = Path(root)
        self.classes = sorted(d.name for d in root.iterdir() if d.is_dir())
        self.items = []
        for i, c in enumerate(self.classes):
            for f in sorted((root / c).iterdir()):
                if f.suffix in IMG_EXT:
                    self.items.append((f, i))
        self.train, self.args = train, args

    def __len__(self):
        return len(self.items)

    def __getitem__(self, i):
        from PIL import Image
        import random
        path, y = self.items[i]
        img = Image.open(path).convert("RGB")
        a = self.args
        interp = {"bilinear": Image.BILINEAR, "bicubic": Image.BICUBIC, "nearest": Image.NEAREST}.get(
            a.interpolation, Image.BILINEAR)
        if self.train:  # RandomResizedCrop(scale .08-1, ratio 3/4-4/3) + horizontal flip
            W, H = img.size
            for _ in range(10):
                area = W * H * random.uniform(0.08, 1.0)
                ar = random.uniform(3 / 4, 4 / 3)
                w, h = int(round((area * ar) ** 0.5)), int(round((area / ar) ** 0.5))
                if 0 < w <= W and 0 < h <= H:
                    x0, y0 = random.randint(0, W - w), random.randint(0, H - h)
                    break
            else:
                w, h = min(W, H), min(W, H)
                x0, y0 = (W - w) // 2, (H - h) // 2
            img = img.crop((x0, y0, x0 + w, y0 + h)).resize((a.train_crop_size,) * 2, interp)
            if random.random() < 0.5:
                img = img.transpose(Image.FLIP_LEFT_RIGHT)
        else:
            W, H = img.size
            s = a.val_resize_size / min(W, H)
            img = img.resize((max(1, round(W * s)), max(1, round(H * s))), interp)
            W, H = img.size
            c = a.val_crop_size
            img = img.crop(((W - c) // 2, (H - c) // 2, (W - c) // 2 + c, (H - c) // 2 + c))
        import numpy as np
        x = torch.from_numpy(np.asarray(img, dtype=np.float32) / 255.0).permute(2, 0, 1)
        x = (x - torch.tensor(MEAN)[:, None, None]) / torch.tensor(STD)[:, None, None]
        return x, y


class Synthetic(torch.utils.data.Dataset):
    def __init__(self, n, size, classes):
        self.n, self.size, self.classes = n, size, classes

    def __len__(self):
        return self.n

    def __getitem__(self, i):
        g = torch.Generator().manual_seed(i)
        return torch.randn(3, self.size, self.size, generator=g), int(torch.randint(0, self.classes, (1,),
                                                                                      generator=g))


def prepare_val(data_dir: Path, labels_csv: Path):
    """LOC_val_solution.csv (ImageId, 'nXXXX x y ...') -> val/<wnid>/<img>."""
    val = Path(data_dir) / "val"
    with open(labels_csv) as f:
        for row in csv.DictReader(f):
            wnid = row["PredictionString"].split()[0]
            src = val / f"{row['ImageId']}.JPEG"
            if src.exists():
                (val / wnid).mkdir(exist_ok=True)
                shutil.move(str(src), str(val / wnid / src.name))


def accuracy(output, target, topk=(1, 5)):
    maxk = min(max(topk), output.shape[1])
    _, pred = output.topk(maxk, 1, True, True)
    correct = pred.t().eq(target.view(1, -1))
    return [correct[:min(k, maxk)].reshape(-1).float().sum() for k in topk]


# ----------------------------------------------------------------- train
def main(argv=None):
    from ..models.resnet import resnet50
    from ..obs.metrics import MetricsSink
    args = build_parser().parse_args(argv)
    if args.prepare_val:
        prepare_val(args.data_dir, args.val_labels)
        return {}
    use_cuda = torch.cuda.is_available() and not args.no_cuda
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", max(args.local_rank, 0)))
    from ..parallel import shared_gpu
    shared = use_cuda and shared_gpu.enabled()  # rehearsal: all ranks on cuda:0, gloo (parallel/shared_gpu.py)
    if use_cuda:
        torch.cuda.set_device(0 if shared else local % torch.cuda.device_count())
    dev = torch.device("cuda", torch.cuda.current_device()) if use_cuda else torch.device("cpu")
    if world > 1 and not dist.is_initialized():
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        dist.init_process_group(backend="gloo" if shared else (args.backend or ("nccl" if use_cuda else "gloo")))
        if shared:
            shared_gpu.install()
    rank = dist.get_rank() if dist.is_initialized() else 0
    torch.manual_seed(args.seed)
    if args.synthetic:
        train_ds = Synthetic(args.synthetic, args.train_crop_size, args.num_classes)
        val_ds = Synthetic(max(args.synthetic // 4, 1), args.val_crop_size, args.num_classes)
    else:
        train_ds = ImageFolder(args.data_dir / "train", True, args)
        val_ds = ImageFolder(args.data_dir / "val", False, args)
    from torch.utils.data import DataLoader, DistributedSampler
    tr_s = DistributedSampler(train_ds, num_replicas=world, rank=rank, shuffle=True, seed=args.seed)
    va_s = DistributedSampler(val_ds, num_replicas=world, rank=rank, shuffle=False)
    tl = DataLoader(train_ds, batch_size=args.batch_size, sampler=tr_s, num_workers=args.workers,
                    pin_memory=use_cuda, drop_last=True, persistent_workers=args.workers > 0)
    vl = DataLoader(val_ds, batch_size=args.batch_size, sampler=va_s, num_workers=args.workers, pin_memory=use_cuda)
    model = resnet50(args.num_classes).to(dev)
    if use_cuda:
        from ..utils import miopen
        miopen.configure()  # keep MIOpen's naive NHWC solvers out of the conv search
        model = model.to(memory_format=torch.channels_last)
    adasum = args.use_adasum and world > 1
    # GPU: average inside the node, Adasum across nodes (Horovod's NCCL build); CPU: flat Adasum
    local = local_size(world) if use_cuda else 1
    if adasum and (world // local) & (world // local - 1):
        print(f"[resnet] --use-adasum needs a power-of-two Adasum group (got {world // local}); averaging instead",
              flush=True)
        adasum = False
    if world > 1:
        model = nn.parallel.DistributedDataParallel(model, device_ids=[dev.index] if use_cuda else None,
                                                    bucket_cap_mb=args.bucket_mb, gradient_as_bucket_view=True)
        if adasum:
            lg, cg = adasum_groups(world, rank, local)
            model.register_comm_hook(state=AdasumState(cg, args.fp16_allreduce, lg), hook=adasum_hook)
        elif args.fp16_allreduce or args.gradient_predivide_factor != 1.0 or shared:
            # (shared-GPU rehearsal: the hook's dist.all_reduce is the host-staged one)
            model.register_comm_hook(state=(dist.group.WORLD, args.fp16_allreduce, args.gradient_predivide_factor),
                                     hook=_compressed_allreduce_hook)
    # Horovod's LR scaler: x world for averaging, 1 for Adasum, x local size for GPU Adasum
    # (resnet50_horovod.py:115-123)
    opt = torch.optim.SGD(model.parameters(), lr=args.lr * (local if adasum else world), momentum=args.momentum)
    sink = MetricsSink(str(args.log_dir), args.wandb_run or "resnet50",
                       project=args.wandb_project or "resnet50-imagenet", enabled=rank == 0)
    amp = args.use_mixed_precision and use_cuda
    step, t_start = 0, time.perf_counter()
    last = {}
    for epoch in range(1, args.epochs + 1):
        model.train()
        tr_s.set_epoch(epoch)
        for bi, (x, y) in enumerate(tl):
            t0 = time.perf_counter()
            x = x.to(dev, non_blocking=True)
            y = y.to(dev, non_blocking=True)
            if use_cuda:
                x = x.contiguous(memory_format=torch.channels_last)
            opt.zero_grad(set_to_none=True)
            with torch.autocast(dev.type, dtype=torch.bfloat16, enabled=amp):
                out = model(x)
                loss = F.cross_entropy(out.float(), y)
            loss.backward()
            opt.step()
            step += 1
            if bi % args.log_interval == 0:
                lv = float(loss)
                dt = time.perf_counter() - t0
                if rank == 0:
                    print(f"Train Epoch: {epoch} [{bi * len(x)}/{len(tr_s)} ({100. * bi / max(len(tl), 1):.0f}%)]"
                          f"\tLoss: {lv:.6f}", flush=True)
                    sink.log({"train/loss": lv, "train/epoch": epoch, "train/step": step,
                              "train/samples_seen": step * len(x) * world,
                              "perf/rank_samples_per_second": len(x) / dt}, step=step)
            if args.max_steps and step >= args.max_steps:
                break
        last = evaluate(model, vl, va_s, dev, world, amp)
        if rank == 0:
            print(f"Test Epoch: {epoch}\tloss={last['loss']:.4f}\tAcc@1={last['acc1']:.3f}\tAcc@5={last['acc5']:.3f}",
                  flush=True)
            sink.log({"test/loss": last["loss"], "test/epoch": epoch, "test/acc1": last["acc1"],
                      "test/acc5": last["acc5"]}, step=step)
        if args.max_steps and step >= args.max_steps:
            break
    if rank == 0:
        print(f"Training time: {time.perf_counter() - t_start:0.3f}s")
        if args.model_dir:
            args.model_dir.mkdir(parents=True, exist_ok=True)
            sd = (model.module if hasattr(model, "module") else model).state_dict()
            torch.save(sd, args.model_dir / "resnet50_imagenet.pt")
        sink.close()
    if dist.is_initialized():
        dist.barrier()
    return {"steps": step, **last}


@torch.no_grad()
def evaluate(model, loader, sampler, dev, world, amp):
    model.eval()
    tot = torch.zeros(4, device=dev, dtype=torch.float64)  # loss sum, acc1, acc5, n
    for x, y in loader:
        x, y = x.to(dev), y.to(dev)
        with torch.autocast(dev.type, dtype=torch.bfloat16, enabled=amp):
            out = model(x).float()
        a1, a5 = accuracy(out, y)
        tot += torch.stack([F.cross_entropy(out, y, reduction="sum"), a1, a5,
                            torch.tensor(float(len(y)), device=dev)]).double()
    if world > 1:
        dist.all_reduce(tot)
    n = max(float(tot[3]), 1.0)
    return {"loss": float(tot[0]) / n, "acc1": 100.0 * float(tot[1]) / n, "acc5": 100.0 * float(tot[2]) / n}


def _compressed_allreduce_hook(state, bucket):
    """Horovod's fp16 compression / predivide factor as a DDP comm hook: bf16
    wire format on MI355X (same bytes as fp16, no overflow), mean over ranks."""
    group, compress, predivide = state
    world = dist.get_world_size(group)
    buf = bucket.buffer()
    t = buf.to(torch.bfloat16) if compress else buf.clone()
    t.div_(predivide)
    fut = dist.all_reduce(t, group=group, async_op=True).get_future()

    def done(f):
        r = f.value()[0]
        buf.copy_(r.to(buf.dtype).mul_(predivide / world))
        return buf
    return fut.then(done)


class AdasumState:
    """``group``: the ranks combined with Adasum; ``local_group`` (hierarchical form): the ranks
    averaged first (one node), None for flat Adasum."""

    def __init__(self, group, compress: bool = False, local_group=None):
        self.group, self.compress, self.local_group = group, compress, local_group
        self.segments: dict = {}  # bucket index -> (segment ids, n tensors)


def local_size(world: int) -> int:
    """GPUs per node: torchrun's LOCAL_WORLD_SIZE (Horovod's hvd.local_size()), else all ranks."""
    n = int(os.environ.get("LOCAL_WORLD_SIZE", world))
    return n if n > 0 and world % n == 0 else world


def adasum_groups(world: int, rank: int, local: int):
    """(local group, cross group) of ``rank`` for hierarchical Adasum: nodes are runs of ``local``
    consecutive ranks; the cross group holds the ranks of equal local rank. Every rank creates
    every group (dist.new_group is collective); a size-1 group is returned as None."""
    lg = cg = None
    for n in range(world // local):
        ranks = list(range(n * local, (n + 1) * local))
        g = dist.new_group(ranks) if local > 1 else None
        if rank in ranks:
            lg = g
    for lr in range(local):
        ranks = list(range(lr, world, local))
        g = dist.new_group(ranks) if len(ranks) > 1 else None
        if rank in ranks:
            cg = g
    return lg, cg


def adasum_pair(a: torch.Tensor, b: torch.Tensor, seg: torch.Tensor, n: int) -> torch.Tensor:
    """Adasum of two flat gradient buffers, coefficients per tensor segment
    (Maleki et al., Horovod's op=hvd.Adasum): (1 - a.b / 2|a|^2) a + (1 - a.b / 2|b|^2) b.
    Symmetric in (a, b), so both partners of a pair compute the same bits."""
    af, bf = a.float(), b.float()
    dot = torch.zeros(n, device=a.device, dtype=torch.float64).index_add_(0, seg, (af * bf).double())
    na = torch.zeros(n, device=a.device, dtype=torch.float64).index_add_(0, seg, (af * af).double())
    nb = torch.zeros(n, device=a.device, dtype=torch.float64).index_add_(0, seg, (bf * bf).double())
    ca = torch.where(na > 0, 1.0 - dot / (2.0 * na), torch.ones_like(na)).float()[seg]
    cb = torch.where(nb > 0, 1.0 - dot / (2.0 * nb), torch.ones_like(nb)).float()[seg]
    return (ca * af + cb * bf).to(a.dtype)


def adasum_allreduce(buf: torch.Tensor, seg: torch.Tensor, n: int, group=None, compress: bool = False):
    """In-place Adasum over all ranks of ``group`` (power-of-two size):
    recursive doubling -- at level l every rank swaps its running result with
    rank ^ 2^l and both combine the pair -- so after log2(W) exchanges every
    rank holds Adasum(Adasum(g0, g1), Adasum(g2, g3)) ... in the same bits."""
    world, rank = dist.get_world_size(group), dist.get_rank(group)
    cur = buf.to(torch.bfloat16) if compress else buf.clone()
    lvl = 1
    while lvl < world:
        peer = rank ^ lvl
        other = torch.empty_like(cur)
        gpeer = dist.get_global_rank(group, peer) if group is not None and group != dist.group.WORLD else peer
        ops = [dist.P2POp(dist.isend, cur, gpeer, group), dist.P2POp(dist.irecv, other, gpeer, group)]
        for w in dist.batch_isend_irecv(ops):
            w.wait()
        # lower rank's buffer first: both partners evaluate the identical expression
        cur = adasum_pair(cur, other, seg, n) if rank < peer else adasum_pair(other, cur, seg, n)
        lvl <<= 1
    buf.copy_(cur.to(buf.dtype))
    return buf


def hierarchical_adasum(buf: torch.Tensor, seg: torch.Tensor, n: int, local_group=None, cross_group=None,
                        compress: bool = False):
    """Average over ``local_group`` (skipped when None), then Adasum over ``cross_group``
    (skipped when None): Horovod's GPU Adasum, node-local reduction + cross-node Adasum."""
    if local_group is not None:
        dist.all_reduce(buf, group=local_group)
        buf.div_(dist.get_world_size(local_group))
    if cross_group is not None:
        adasum_allreduce(buf, seg, n, cross_group, compress)
    return buf


def adasum_hook(state: AdasumState, bucket):
    """DDP comm hook: the bucket's flat gradient is combined with Adasum, one
    coefficient pair per parameter tensor of the bucket."""
    buf = bucket.buffer()
    key = bucket.index()
    seg = state.segments.get(key)
    if seg is None or seg[0].numel() != buf.numel():
        ids = [torch.full((g.numel(),), i, dtype=torch.long) for i, g in enumerate(bucket.gradients())]
        seg = (torch.cat(ids).to(buf.device), len(ids))
        state.segments[key] = seg
    hierarchical_adasum(buf, seg[0], seg[1], state.local_group, state.group, state.compress)
    fut = torch.futures.Future()
    fut.set_result(buf)
    return fut


if __name__ == "__main__":
    main()
