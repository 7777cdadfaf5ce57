"""HF-Trainer-style checkpoint directories + the ``.ready.txt`` sentinel.

Layout written under ``{output_path}/results-{run_name}/``
(finetuner-workflow/finetuner/finetuner.py:345-347, 1016-1018, 1055-1062):

    checkpoint-{step}/
        config.json, model.safetensors[.index.json + shards]   (HF names)
        trainer_state.json          global_step, epoch, log_history, schedule
        training_args.json          the CLI namespace
        optimizer/rank-{r:05d}.safetensors   fp32 master/exp_avg/exp_avg_sq shard
        optimizer/meta.json         world size, layout size, ZeRO stage
        rng_state_{r}.pth           torch / cuda / numpy / python RNG (own file)
    final/  model + tokenizer + .ready.txt

Resume picks the largest numeric ``checkpoint-N`` and *skips* entries without
a numeric suffix (the reference's scan silently disabled resume when e.g.
``final/`` existed: finetuner.py:350-357 -- SURVEY §7.6).
"""
from __future__ import annotations

import json
import os
import random
import re
import time

import numpy as np
import torch

_CKPT = re.compile(r"^checkpoint-(\d+)$")


def checkpoint_complete(path: str) -> bool:
    """A checkpoint dir is complete when it carries no ``.incomplete`` marker,
    or when every rank named in the marker has written its ``.done-rank{r}``
    (the async writers finished even if the process died before the next
    save / the final barrier removed the marker)."""
    inc = os.path.join(path, ".incomplete")
    if not os.path.exists(inc):
        return True
    try:
        with open(inc) as f:
            world = int(f.read().strip() or "0")
    except (OSError, ValueError):
        return False
    return world > 0 and all(os.path.exists(os.path.join(path, f".done-rank{r}")) for r in range(world))


def find_last_checkpoint(output_dir: str) -> str | None:
    try:
        names = os.listdir(output_dir)
    except FileNotFoundError:
        return None
    best = None
    for n in names:
        m = _CKPT.match(n)
        if m and os.path.isdir(os.path.join(output_dir, n)) and checkpoint_complete(os.path.join(output_dir, n)):
            step = int(m.group(1))
            if best is None or step > best[0]:
                best = (step, n)
    return os.path.join(output_dir, best[1]) if best else None


def write_ready(path: str):
    os.makedirs(path, exist_ok=True)
    open(os.path.join(path, ".ready.txt"), "a").close()


def wait_ready(path: str, timeout_s: float = 3600, poll_s: float = 5.0) -> bool:
    """Poll for ``.ready.txt`` like the BLOOM / DALL-E predictors
    (online-inference/bloom-176b/model/bloom.py:79-90)."""
    t0 = time.time()
    f = os.path.join(path, ".ready.txt")
    while not os.path.exists(f):
        if time.time() - t0 > timeout_s:
            return False
        time.sleep(poll_s)
    return True


def _rng_state():
    st = {"torch": torch.get_rng_state(), "numpy": np.random.get_state()[1].astype(np.int64),
          "python": random.getstate()[1]}
    if torch.cuda.is_available():
        st["cuda"] = torch.cuda.get_rng_state()
    return st


def save_checkpoint(ckpt_dir: str, model, engine, trainer_state: dict, args_dict: dict | None = None,
                    tokenizer=None, rank: int = 0, world: int = 1, barrier=None):
    """Synchronous save (ZeRO-3 callers wrap it in ``engine.gathered()``)."""
    from safetensors.torch import save_file

    from .hf import save_pretrained

    os.makedirs(os.path.join(ckpt_dir, "optimizer"), exist_ok=True)
    if rank == 0:
        save_pretrained(model, ckpt_dir)
        if tokenizer is not None:
            tokenizer.save_pretrained(ckpt_dir)
        with open(os.path.join(ckpt_dir, "trainer_state.json"), "w") as f:
            json.dump(trainer_state, f, indent=2, default=str)
        if args_dict is not None:
            with open(os.path.join(ckpt_dir, "training_args.json"), "w") as f:
                json.dump(args_dict, f, indent=2, default=str)
    if engine is not None:
        st = engine.optimizer_state()
        tensors = {"master": st["master"].detach().cpu(), "exp_avg": st["exp_avg"].detach().cpu(),
                   "exp_avg_sq": st["exp_avg_sq"].detach().cpu()}
        save_file(tensors, os.path.join(ckpt_dir, "optimizer", f"rank-{rank:05d}.safetensors"))
        if rank == 0:
            with open(os.path.join(ckpt_dir, "optimizer", "meta.json"), "w") as f:
                json.dump({"world": st["world"], "total": st["total"], "step": st["step"],
                           "zero_stage": st["zero_stage"], "lr": st["lr"], "layout": st["layout"]}, f)
    rs = _rng_state()
    torch.save({k: (torch.as_tensor(v) if not isinstance(v, torch.Tensor) else v) for k, v in rs.items()},
               os.path.join(ckpt_dir, f"rng_state_{rank}.pth"))
    if barrier is not None:
        barrier()


class _Snapshot:
    """Host copy of a model/engine, reusing pinned buffers between saves."""

    def __init__(self):
        self.bufs: dict = {}

    def take(self, name: str, t: torch.Tensor) -> torch.Tensor:
        b = self.bufs.get(name)
        if b is None or b.shape != t.shape or b.dtype != t.dtype:
            b = torch.empty(t.shape, dtype=t.dtype, pin_memory=t.is_cuda)
            self.bufs[name] = b
        b.copy_(t.detach(), non_blocking=True)
        return b


class AsyncCheckpointWriter:
    """checkpoint I/O off the training critical path.

    ``save`` snapshots parameters, optimizer shard and RNG into reused pinned
    host buffers (a D2H copy at ~50 GB/s, then one sync), and a background
    thread serialises them to ``checkpoint-N/`` (safetensors + JSON) while
    training continues; the next ``save`` (or ``wait``) joins the previous
    writer first, so at most one snapshot is in flight."""

    def __init__(self, rank: int = 0):
        self._snap = _Snapshot()  # one set of pinned buffers: the previous writer is joined first
        self._thread = None
        self._err = None
        self._pending = None
        self.rank = rank

    def wait(self, barrier=None):
        """Join this rank's writer; with ``barrier`` (all ranks) mark the pending
        checkpoint complete (rank 0 removes its ``.incomplete`` sentinel)."""
        if self._thread is not None:
            self._thread.join()
            self._thread = None
        if self._err is not None:
            e, self._err = self._err, None
            raise e
        if self._pending is not None:
            if barrier is not None:
                barrier()
            if self.rank == 0:
                try:
                    os.remove(os.path.join(self._pending, ".incomplete"))
                except FileNotFoundError:
                    pass
            self._pending = None

    def save(self, ckpt_dir: str, model, engine, trainer_state: dict, args_dict: dict | None = None,
             tokenizer=None, rank: int = 0, world: int = 1, barrier=None):
        import copy
        import threading
        self.rank = rank
        self.wait(barrier)
        snap = self._snap
        # only rank 0 writes the model files: other ranks snapshot just their optimizer shard + RNG
        # (8 ranks x a bf16 replica in pinned host memory would be ~96 GB for GPT-J)
        params = {k: snap.take("p." + k, v) for k, v in model.state_dict().items()} if rank == 0 else None
        opt = None
        if engine is not None:
            st = engine.optimizer_state()
            opt = ({k: snap.take("o." + k, st[k]) for k in ("master", "exp_avg", "exp_avg_sq")},
                   {k: st[k] for k in ("world", "total", "step", "zero_stage", "lr", "layout")})
        if torch.cuda.is_available():
            torch.cuda.synchronize()
        rng = _rng_state()
        state = copy.deepcopy(trainer_state)
        os.makedirs(os.path.join(ckpt_dir, "optimizer"), exist_ok=True)
        # every rank marks the dir incomplete before its writer starts (resume skips it until all
        # ranks' .done-rank markers exist or the post-save barrier removed the marker)
        with open(os.path.join(ckpt_dir, ".incomplete"), "w") as f:
            f.write(str(world))
        if rank == 0 and tokenizer is not None:
            tokenizer.save_pretrained(ckpt_dir)
        try:  # a re-save of the same step starts from no done markers
            os.remove(os.path.join(ckpt_dir, f".done-rank{rank}"))
        except FileNotFoundError:
            pass
        self._pending = ckpt_dir

        def write():
            try:
                _write_checkpoint(ckpt_dir, model.cfg, params, opt, state, args_dict, rng, rank)
                with open(os.path.join(ckpt_dir, f".done-rank{rank}"), "w") as f:
                    f.write("ok")
            except Exception as e:  # noqa: BLE001 -- surfaced on the next wait()/save()
                self._err = e
        self._thread = threading.Thread(target=write, name="ckpt-writer", daemon=False)
        self._thread.start()


def _write_checkpoint(ckpt_dir, cfg, params, opt, trainer_state, args_dict, rng, rank):
    from safetensors.torch import save_file

    from ..models.hf_convert import native_to_hf
    if rank == 0:
        hf = native_to_hf({k: v for k, v in params.items() if not k.endswith("alibi")}, cfg)
        save_file({k: v.contiguous() for k, v in hf.items()}, os.path.join(ckpt_dir, "model.safetensors"),
                  metadata={"format": "pt"})
        with open(os.path.join(ckpt_dir, "config.json"), "w") as f:
            json.dump(cfg.to_hf(), f, indent=2)
        with open(os.path.join(ckpt_dir, "trainer_state.json"), "w") as f:
            json.dump(trainer_state, f, indent=2, default=str)
        if args_dict is not None:
            with open(os.path.join(ckpt_dir, "training_args.json"), "w") as f:
                json.dump(args_dict, f, indent=2, default=str)
    if opt is not None:
        tensors, meta = opt
        save_file(tensors, os.path.join(ckpt_dir, "optimizer", f"rank-{rank:05d}.safetensors"))
        if rank == 0:
            with open(os.path.join(ckpt_dir, "optimizer", "meta.json"), "w") as f:
                json.dump(meta, f)
    torch.save({k: (torch.as_tensor(v) if not isinstance(v, torch.Tensor) else v) for k, v in rng.items()},
               os.path.join(ckpt_dir, f"rng_state_{rank}.pth"))


def load_checkpoint(ckpt_dir: str, model, engine, rank: int = 0) -> dict:
    from safetensors.torch import load_file

    from ..models.hf_convert import hf_to_native
    from .hf import read_hf_state_dict

    if engine is None or not getattr(engine, "part_params", False):
        # (ZeRO-3: the params are this rank's bf16 shard, re-derived from the fp32 master below)
        sd = hf_to_native(read_hf_state_dict(ckpt_dir), model.cfg)
        with torch.no_grad():
            own = model.state_dict()
            for k, v in sd.items():
                if k in own:
                    own[k].copy_(v.to(own[k].dtype))
    if engine is not None:
        with open(os.path.join(ckpt_dir, "optimizer", "meta.json")) as f:
            meta = json.load(f)
        t = load_file(os.path.join(ckpt_dir, "optimizer", f"rank-{rank:05d}.safetensors"))
        dev = engine.opt.master.device
        engine.load_optimizer_state({"master": t["master"].to(dev), "exp_avg": t["exp_avg"].to(dev),
                                     "exp_avg_sq": t["exp_avg_sq"].to(dev), "step": meta["step"],
                                     "lr": meta.get("lr"), "world": meta["world"],
                                     "total": meta["total"], "zero_stage": meta.get("zero_stage"),
                                     **({"layout": meta["layout"]} if "layout" in meta else {})})
    p = os.path.join(ckpt_dir, f"rng_state_{rank}.pth")
    if os.path.exists(p):
        rs = torch.load(p, weights_only=True)
        torch.set_rng_state(rs["torch"])
        if "cuda" in rs and torch.cuda.is_available():
            torch.cuda.set_rng_state(rs["cuda"])
    with open(os.path.join(ckpt_dir, "trainer_state.json")) as f:
        return json.load(f)
