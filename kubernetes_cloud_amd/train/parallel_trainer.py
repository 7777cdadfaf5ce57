"""3D-parallel causal-LM trainer: TP x PP x DP (T12).

Replaces the reference's GPT-NeoX-20B MPIJob (external gpt-neox image, PP=4,
TP=2, ZeRO-1, micro-batch 8, GAS 96, Adam .9/.95, clip 1.0, cosine LR,
activation checkpointing: kubeflow/training-operator/gpt-neox/
04-finetune-workflow.yaml:171-304) with this framework's own pieces:

    torchrun --nproc-per-node 8 -m kubernetes_cloud_amd.train.parallel_trainer \
        --model /ckpt/neox-20b --dataset /data/hn.tokens --tp 2 --pp 4 ...

Rank layout (tp fastest, then pp, then dp) keeps a TP group on adjacent GPUs
of one node, i.e. on direct xGMI links, where its 4 all-reduces per layer per
micro-batch run; pipeline p2p and the once-per-step DP all-reduce tolerate the
slower paths. Every rank holds only its (stage, TP shard) of the weights, and
the optimizer state is ZeRO-1 sharded over the DP group (``--zero-stage 1``,
the reference's setting): per-bucket reduce-scatter over DP in the last
micro-batch's backward, the clip norm summed over DP then over the
model-parallel group with TP-replicated params counted once.

Checkpoints: ``{output}/checkpoint-{step}/mp_rank_{tp:02d}_{pp:03d}.safetensors``
(written by dp rank 0 of each shard) + ``meta.json``; ``consolidate`` rebuilds
a full HF directory from them (for serving / the finetuner).
"""
from __future__ import annotations

import argparse
import json
import os
import time

import torch
import torch.distributed as dist

from ..parallel.pipeline import P2P, build_stage, one_f_one_b, split_layers, tie_embedding_grads
from ..parallel.tensor_parallel import shard_native_tensor, tp_convert_
from .engine import TrainEngine
from .optim import lr_at


def build_parser():
    p = argparse.ArgumentParser(description="TP x PP x DP causal-LM trainer")
    p.add_argument("--model", required=True, help="HF checkpoint dir, or preset name with --random-init")
    p.add_argument("--random-init", action="store_true")
    p.add_argument("--layers", type=int, default=0, help="override layer count (tests/benches)")
    p.add_argument("--dataset", default="", help=".tokens file (uint16); empty = synthetic tokens")
    p.add_argument("--output-path", default="")
    p.add_argument("--tp", type=int, default=1)
    p.add_argument("--pp", type=int, default=1)
    p.add_argument("--micro-batch", type=int, default=1)
    p.add_argument("--gradients", type=int, default=1, help="micro-batches per optimizer step (GAS)")
    p.add_argument("--seq-len", type=int, default=2048)
    p.add_argument("--zero-stage", type=int, default=1, choices=(0, 1, 2),
                   help="ZeRO stage over the data-parallel group (NeoX: 1, 04-finetune-workflow.yaml:236-244)")
    p.add_argument("--gradient-checkpointing", action="store_true")
    p.add_argument("--lr", type=float, default=6e-5)
    p.add_argument("--min-lr", type=float, default=0.0)
    p.add_argument("--betas", type=float, nargs=2, default=(0.9, 0.95))
    p.add_argument("--eps", type=float, default=1e-8)
    p.add_argument("--weight-decay", type=float, default=0.01)
    p.add_argument("--max-grad-norm", type=float, default=1.0)
    p.add_argument("--lr-schedule", default="cosine", choices=["cosine", "linear", "constant"])
    p.add_argument("--warmup-ratio", type=float, default=0.01)
    p.add_argument("--epochs", type=int, default=1)
    p.add_argument("--max-steps", type=int, default=0)
    p.add_argument("--save-steps", type=int, default=0)
    p.add_argument("--seed", type=int, default=42)
    p.add_argument("--fp32", action="store_true",
                   help="fp32 parameters and math on the GPU (parity references; the native kernels are bf16)")
    p.add_argument("--log-dir", default="")
    p.add_argument("--local_rank", "--local-rank", type=int, default=-1,
                   help="appended by the DeepSpeed-style launcher (kubernetes_cloud_amd.launch); LOCAL_RANK wins")
    return p


class Topology:
    def __init__(self, tp: int, pp: int):
        self.world = dist.get_world_size() if dist.is_initialized() else 1
        self.rank = dist.get_rank() if dist.is_initialized() else 0
        if self.world % (tp * pp):
            raise ValueError(f"world {self.world} not divisible by tp*pp={tp * pp}")
        self.tp, self.pp, self.dp = tp, pp, self.world // (tp * pp)
        r = self.rank
        self.tp_idx, self.pp_idx, self.dp_idx = r % tp, (r // tp) % pp, r // (tp * pp)
        self.tp_group = self.dp_group = self.mp_group = self.embed_group = None
        if self.world == 1:
            return

        def R(d, p, t):
            return d * tp * pp + p * tp + t
        for d in range(self.dp):  # every rank creates every group, same order
            for p in range(pp):
                g = dist.new_group([R(d, p, t) for t in range(tp)])
                if d == self.dp_idx and p == self.pp_idx:
                    self.tp_group = g
        for p in range(pp):
            for t in range(tp):
                g = dist.new_group([R(d, p, t) for d in range(self.dp)])
                if p == self.pp_idx and t == self.tp_idx:
                    self.dp_group = g
        for d in range(self.dp):
            g = dist.new_group([R(d, p, t) for p in range(pp) for t in range(tp)])
            if d == self.dp_idx:
                self.mp_group = g
        if pp > 1:
            for d in range(self.dp):
                for t in range(tp):
                    g = dist.new_group([R(d, 0, t), R(d, pp - 1, t)])
                    if d == self.dp_idx and t == self.tp_idx and self.pp_idx in (0, pp - 1):
                        self.embed_group = g
        self.prev = R(self.dp_idx, self.pp_idx - 1, self.tp_idx) if self.pp_idx > 0 else None
        self.next = R(self.dp_idx, self.pp_idx + 1, self.tp_idx) if self.pp_idx < pp - 1 else None


def stage_to_full_name(name: str, lo: int) -> str:
    if name.startswith("h."):
        i, rest = name[2:].split(".", 1)
        return f"h.{int(i) + lo}.{rest}"
    if name == "head_weight":
        return "wte.weight"
    return name


def build_model_shard(args, topo: Topology, device, dtype):
    from ..models.causal_lm import CausalLM, alibi_slopes
    from ..models.config import LMConfig, preset
    cfg = preset(args.model) if args.random_init else LMConfig.from_pretrained(args.model)
    if args.layers:
        cfg.n_layers = args.layers
    if cfg.tie_embeddings and topo.tp > 1 and topo.pp > 1:
        raise NotImplementedError("tied embeddings with TP and PP together (use TP or PP for GPT-2/BLOOM)")
    with torch.device("meta"):
        full = CausalLM(cfg)
    if topo.tp > 1:
        tp_convert_(full, topo.tp_idx, topo.tp, topo.tp_group)
    stage = build_stage(full, topo.pp_idx, topo.pp)
    stage = stage.to_empty(device=device).to(dtype)
    if cfg.alibi:
        Hl = cfg.n_heads // topo.tp
        for blk in stage.h:
            blk.attn.alibi = alibi_slopes(cfg.n_heads)[topo.tp_idx * Hl:(topo.tp_idx + 1) * Hl].to(device)
    with torch.no_grad():
        if args.random_init:
            g = torch.Generator(device=device).manual_seed(args.seed + 1000 * topo.pp_idx + topo.tp_idx)
            for n, p in stage.named_parameters():
                if p.dim() >= 2:
                    p.normal_(0.0, 0.02, generator=g)
                else:
                    p.fill_(1.0 if n.endswith("weight") else 0.0)
        else:
            from ..models.hf_convert import hf_to_native_plan, prefixed_getter
            from ..parallel.tensor_parallel import _LazySafetensors
            sd = _LazySafetensors(args.model)
            plan = hf_to_native_plan(cfg, prefixed_getter(sd), tuple(sd.keys()))
            for n, p in stage.named_parameters():
                fn = stage_to_full_name(n, stage.lo)
                full_t = plan[fn]()
                shard = shard_native_tensor(fn, full_t, cfg, topo.tp_idx, topo.tp) if topo.tp > 1 else full_t
                p.copy_(shard.to(p.dtype))
    if not cfg.tie_embeddings:
        topo.embed_group = None  # (the group exists on every rank; unused for untied models)
    if topo.embed_group is not None:
        # make the two copies of a tied embedding bit-identical
        src_rank = topo.rank - (topo.pp - 1) * topo.tp if topo.pp_idx == topo.pp - 1 else topo.rank
        w = stage.wte.weight if stage.first else stage.head_weight
        dist.broadcast(w.data, src=src_rank, group=topo.embed_group)
    stage.gradient_checkpointing = args.gradient_checkpointing
    return cfg, stage


def replicated_param_names(stage) -> set:
    """Params that every TP rank holds in full (counted once in the clip norm)."""
    from ..parallel.tensor_parallel import ColumnParallelLinear, ParallelLMHead, RowParallelLinear
    out = set()
    sharded = set()
    for mname, mod in stage.named_modules():
        if isinstance(mod, (ColumnParallelLinear, ParallelLMHead)):
            for pn, _ in mod.named_parameters(recurse=False):
                sharded.add(f"{mname}.{pn}")
        if isinstance(mod, RowParallelLinear):
            sharded.add(f"{mname}.weight")
    for n, _ in stage.named_parameters():
        if n not in sharded:
            out.add(n)
    return out


def data_stream(args, cfg, topo: Topology, device):
    """Per-DP-replica micro-batches [mb, S] (same on every stage/TP rank of a replica)."""
    mb, S, M = args.micro_batch, args.seq_len, args.gradients
    if args.dataset:
        from ..data.tokenized import TokenizedDataset
        ds = TokenizedDataset(args.dataset, S)
        n = len(ds)
        g = torch.Generator().manual_seed(args.seed)
        order = torch.randperm(n, generator=g).tolist()
        per_step = mb * M * topo.dp
        steps = n // per_step
        for ep in range(args.epochs):
            for s in range(steps):
                base = s * per_step + topo.dp_idx * mb * M
                idx = order[base:base + mb * M]
                rows = torch.stack([ds[i][0] for i in idx])
                yield [rows[k * mb:(k + 1) * mb].to(device) for k in range(M)]
    else:
        # synthetic: the step's GLOBAL batch (dp x mb x M rows) from one seeded stream, replica d taking
        # its contiguous share -- a world-1 run with micro-batch dp x mb consumes the same rows per
        # optimizer step, so DP runs compare element-wise against it (tests/test_multirank_train_gpu.py)
        g = torch.Generator().manual_seed(args.seed)
        while True:
            rows = torch.randint(0, cfg.vocab_size, (topo.dp * mb * M, S), generator=g)
            mine = rows[topo.dp_idx * mb * M:(topo.dp_idx + 1) * mb * M]
            yield [mine[k * mb:(k + 1) * mb].to(device) for k in range(M)]


def save_shard(path: str, stage, topo: Topology, step: int, cfg):
    from safetensors.torch import save_file
    os.makedirs(path, exist_ok=True)
    if topo.dp_idx == 0:
        sd = {stage_to_full_name(n, stage.lo): p.detach().contiguous().cpu() for n, p in stage.named_parameters()
              if n != "head_weight"}
        save_file(sd, os.path.join(path, f"mp_rank_{topo.tp_idx:02d}_{topo.pp_idx:03d}.safetensors"))
    if topo.rank == 0:
        with open(os.path.join(path, "meta.json"), "w") as f:
            json.dump({"step": step, "tp": topo.tp, "pp": topo.pp, "config": cfg.to_hf()}, f)


def consolidate(ckpt: str, out_dir: str):
    """Merge TP/PP shards into one HF checkpoint dir (offline, CPU)."""
    from safetensors.torch import load_file

    from ..io.hf import save_pretrained
    from ..models.causal_lm import build_model
    from ..models.config import LMConfig
    with open(os.path.join(ckpt, "meta.json")) as f:
        meta = json.load(f)
    cfg = LMConfig.from_hf(meta["config"])
    tp = meta["tp"]
    parts: dict = {}
    for fn in sorted(os.listdir(ckpt)):
        if fn.startswith("mp_rank_"):
            t = int(fn[8:10])
            for k, v in load_file(os.path.join(ckpt, fn)).items():
                parts.setdefault(k, {})[t] = v
    full = {}
    H, D = cfg.n_heads, cfg.head_dim
    for k, by_t in parts.items():
        sh = [by_t[t] for t in sorted(by_t)]
        if len(sh) == 1 or tp == 1:
            full[k] = sh[0]
        elif k.endswith("attn.qkv.weight") or k.endswith("attn.qkv.bias"):
            Hl = H // tp
            full[k] = torch.cat([s.view(3, Hl, D, *s.shape[1:]) for s in sh], 1).reshape(3 * H * D, *sh[0].shape[1:])
        elif k.endswith("attn.out.weight") or k.endswith("mlp.fc_out.weight"):
            full[k] = torch.cat(sh, 1)
        elif k.endswith("mlp.fc_in.weight") or k.endswith("mlp.fc_in.bias") or k.startswith("lm_head."):
            full[k] = torch.cat(sh, 0)
        else:
            full[k] = sh[0]
    m = build_model(cfg, dtype=next(iter(full.values())).dtype)
    m.load_state_dict(full, strict=False)
    save_pretrained(m, out_dir)
    return out_dir


def main(argv=None):
    from ..obs.metrics import MetricsSink
    from ..parallel.dist import init_distributed
    args = build_parser().parse_args(argv)
    info = init_distributed()
    topo = Topology(args.tp, args.pp)
    dev = torch.device("cuda", torch.cuda.current_device()) if torch.cuda.is_available() else torch.device("cpu")
    dtype = torch.bfloat16 if dev.type == "cuda" and not args.fp32 else torch.float32
    torch.manual_seed(args.seed)
    cfg, stage = build_model_shard(args, topo, dev, dtype)
    stage.train()
    eng = TrainEngine(stage, lr=args.lr, betas=tuple(args.betas), eps=args.eps, weight_decay=args.weight_decay,
                      max_grad_norm=args.max_grad_norm, zero_stage=args.zero_stage, grad_accum=args.gradients,
                      group=topo.dp_group)
    if topo.world > 1:
        rep = {n: topo.tp for n in replicated_param_names(stage)} if topo.tp > 1 else {}
        if getattr(stage, "head_weight", None) is not None:
            rep["head_weight"] = 0  # the first stage's tied copy carries it in the norm
        eng.set_model_parallel(topo.mp_group, rep)
    tie_embedding_grads(eng, stage, topo.embed_group)
    p2p = P2P(topo.prev if topo.world > 1 else None, topo.next if topo.world > 1 else None,
              (args.micro_batch, args.seq_len, cfg.hidden), dtype, dev)
    total = args.max_steps or 10 ** 9
    warm = int(total * args.warmup_ratio) if args.max_steps else 0
    log_rank = (topo.pp - 1) * topo.tp  # dp 0, last stage, tp 0: the rank that holds the loss
    sink = MetricsSink(args.log_dir or os.path.join(args.output_path or ".", "logs"), "parallel-trainer",
                       enabled=topo.rank == log_rank and bool(args.log_dir or args.output_path))
    step, losses = 0, []
    t0 = time.perf_counter()
    for mbs in data_stream(args, cfg, topo, dev):
        lr = lr_at(step, args.lr, total, warm, args.lr_schedule, args.min_lr)
        loss_sum = one_f_one_b(stage, eng, p2p, mbs, topo.pp_idx, topo.pp)
        eng.step(lr)
        step += 1
        if topo.dp > 1:  # the global batch's loss: mean over the data-parallel replicas (every rank joins
            ls = torch.as_tensor(loss_sum, dtype=torch.float32, device=dev).reshape(1)  # its own DP group)
            dist.all_reduce(ls, group=topo.dp_group)
            loss_sum = ls / topo.dp
        losses.append(float(loss_sum / args.gradients))  # meaningful on the last stage only
        if topo.rank == log_rank:
            tok_s = args.micro_batch * args.gradients * args.seq_len * topo.dp * step / (time.perf_counter() - t0)
            sink.log({"train/loss": losses[-1], "train/learning_rate": lr, "train/grad_norm": eng.grad_norm(),
                      "perf/world_tokens_per_second": tok_s}, step=step)
        if args.save_steps and args.output_path and step % args.save_steps == 0:
            save_shard(os.path.join(args.output_path, f"checkpoint-{step}"), stage, topo, step, cfg)
        if args.max_steps and step >= args.max_steps:
            break
    if args.output_path:
        save_shard(os.path.join(args.output_path, f"checkpoint-{step}"), stage, topo, step, cfg)
    sink.close()
    if dist.is_initialized():
        dist.barrier()
    return {"steps": step, "losses": losses, "last_stage": topo.pp_idx == topo.pp - 1, "rank": topo.rank,
            "dt": time.perf_counter() - t0}


if __name__ == "__main__":
    main()
