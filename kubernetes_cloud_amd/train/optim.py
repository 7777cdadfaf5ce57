"""Flat-buffer AdamW (K7), LR schedules (K8) and dynamic loss scaling (K9).

Mirrors the optimizer semantics the reference configures through DeepSpeed /
HF (finetuner-workflow/finetuner/ds_config.json:10-26: AdamW, WarmupLR;
finetuner.py:987-1027: weight_decay, warmup_ratio, linear decay) and the SD
trainer (sd-finetuner/finetuner.py:680-686, 751: AdamW + get_scheduler), but
runs as ONE fused HIP launch over contiguous fp32 buffers:

    master  fp32 [n]   (the ZeRO shard of a rank is a slice of it)
    grad    fp32 [n]   (micro-batch grads accumulated here in fp32)
    exp_avg, exp_avg_sq fp32 [n]
    model_bf16  bf16 [n] (optional: written in the same pass)

The global grad-norm clip and the 1/loss_scale unscale are a device scalar the
kernel reads, so the step never synchronises with the host.
"""
from __future__ import annotations

import math

import torch

from ..ops import _lib


class FlatAdamW:
    def __init__(self, master: torch.Tensor, lr: float = 1e-3, betas=(0.9, 0.999), eps: float = 1e-8,
                 weight_decay: float = 0.0, wd_mask: torch.Tensor | None = None,
                 model_bf16: torch.Tensor | None = None, grad: torch.Tensor | None = None):
        assert master.dtype == torch.float32 and master.dim() == 1
        self.master = master
        self.grad = grad if grad is not None else torch.zeros_like(master)
        self.exp_avg = torch.zeros_like(master)
        self.exp_avg_sq = torch.zeros_like(master)
        self.model_bf16 = model_bf16
        self.lr = lr
        self.betas = betas
        self.eps = eps
        self.weight_decay = weight_decay
        self.wd_mask = wd_mask  # uint8 [n/64]: 1 = apply weight decay to that 64-block
        self.step_count = 0
        dev = master.device
        self._coef = torch.ones(1, device=dev, dtype=torch.float32)
        self._sumsq = torch.zeros(1, device=dev, dtype=torch.float32)
        self._norm = torch.zeros(1, device=dev, dtype=torch.float32)
        self._skip = torch.zeros(1, device=dev, dtype=torch.int32)
        self._ws = torch.empty(1024, device=dev, dtype=torch.float32)
        self.native = master.is_cuda
        if self.native:
            assert master.numel() % 4 == 0, "pad flat buffers to a multiple of 4"
            _lib.require()

    # -- grad norm -------------------------------------------------------
    def local_sumsq(self) -> torch.Tensor:
        """Sum of squares of this rank's grad slice (device scalar, no sync)."""
        if self.native:
            _lib.call("kca_sumsq", self.grad.data_ptr(), self.grad.numel(), self._ws.data_ptr(),
                      self._sumsq.data_ptr(), _lib.stream())
        else:
            self._sumsq.copy_(self.grad.float().pow(2).sum().view(1))
        return self._sumsq

    def set_clip(self, sumsq: torch.Tensor, max_norm: float, inv_loss_scale: float = 1.0):
        """coef = min(1, max_norm/||g||) / loss_scale; skip if non-finite."""
        if self.native:
            _lib.call("kca_clip_coef", sumsq.data_ptr(), float(max_norm), float(inv_loss_scale),
                      self._coef.data_ptr(), self._norm.data_ptr(), self._skip.data_ptr(),
                      _lib.stream())
        else:
            nrm = sumsq.sqrt() * inv_loss_scale
            c = torch.full_like(nrm, inv_loss_scale)
            if max_norm > 0:
                c = torch.where(nrm > max_norm, c * max_norm / (nrm + 1e-6), c)
            self._coef.copy_(c)
            self._norm.copy_(nrm)
            self._skip.copy_((~torch.isfinite(sumsq)).int())

    @property
    def grad_norm(self) -> torch.Tensor:
        return self._norm

    @property
    def skipped(self) -> torch.Tensor:
        return self._skip

    # -- update ------------------------------------------------------------
    def step(self, lr: float | None = None, use_clip: bool = False):
        if lr is not None:
            self.lr = lr
        self.step_count += 1
        b1, b2 = self.betas
        bc1 = 1.0 - b1 ** self.step_count
        bc2 = 1.0 - b2 ** self.step_count
        if self.native:
            # the kernel writes the model copy as bf16; an fp32 model (GPU fp32 training) aliases the
            # master itself (engine: master = flat.float()), any other dtype is copied after
            mb = self.model_bf16
            copy_after = mb is not None and mb.dtype != torch.bfloat16 and mb.data_ptr() != self.master.data_ptr()
            if mb is not None and mb.dtype != torch.bfloat16:
                mb = None
            _lib.call("kca_adamw", self.master.data_ptr(), self.grad.data_ptr(), self.exp_avg.data_ptr(),
                      self.exp_avg_sq.data_ptr(), _lib.ptr(mb), self.master.numel(),
                      _lib.ptr(self.wd_mask), float(self.lr), float(b1), float(b2), float(self.eps),
                      float(self.weight_decay), float(bc1), float(bc2),
                      self._coef.data_ptr() if use_clip else None,
                      self._skip.data_ptr() if use_clip else None, _lib.stream())
            if copy_after:
                self.model_bf16.copy_(self.master)
            return
        if use_clip and bool(self._skip.item()):
            return
        g = self.grad * (self._coef if use_clip else 1.0)
        self.exp_avg.mul_(b1).add_(g, alpha=1 - b1)
        self.exp_avg_sq.mul_(b2).addcmul_(g, g, value=1 - b2)
        denom = (self.exp_avg_sq.sqrt() / math.sqrt(bc2)).add_(self.eps)
        if self.weight_decay:
            if self.wd_mask is None:
                self.master.mul_(1 - self.lr * self.weight_decay)
            else:
                m = self.wd_mask.to(self.master.device).bool().repeat_interleave(64)[: self.master.numel()]
                self.master.mul_(torch.where(m, 1 - self.lr * self.weight_decay, 1.0))
        self.master.addcdiv_(self.exp_avg, denom, value=-self.lr / bc1)
        if self.model_bf16 is not None:
            self.model_bf16.copy_(self.master)

    def state_dict(self):
        return {"exp_avg": self.exp_avg, "exp_avg_sq": self.exp_avg_sq, "step": self.step_count,
                "lr": self.lr, "betas": list(self.betas), "eps": self.eps,
                "weight_decay": self.weight_decay}

    def load_state_dict(self, sd):
        self.exp_avg.copy_(sd["exp_avg"])
        self.exp_avg_sq.copy_(sd["exp_avg_sq"])
        self.step_count = int(sd["step"])
        self.lr = sd.get("lr", self.lr)


class FlatAdamW8bit(FlatAdamW):
    """Block-wise 8-bit AdamW (csrc/kernels/adamw8bit.hip): the bitsandbytes
    AdamW8bit that ``--use_8bit_adam`` selects in the reference SD trainer
    (sd-finetuner-workflow/sd-finetuner/finetuner.py:669-678).

    exp_avg -> int8 codes + fp32 absmax per 2048-element block, exp_avg_sq ->
    uint8 codes + absmax, companded (m = a*sign*(|c|/127)^2, v = a*(c/255)^4)
    so small moments keep their precision: 2 B/param of state instead of 8.
    Master params stay fp32. The CPU path implements the same math in torch.
    """

    BLOCK = 2048

    def __init__(self, master: torch.Tensor, *args, **kw):
        super().__init__(master, *args, **kw)
        n = master.numel()
        nb = (n + self.BLOCK - 1) // self.BLOCK
        dev = master.device
        del self.exp_avg, self.exp_avg_sq
        self.m_codes = torch.zeros(n, device=dev, dtype=torch.int8)
        self.v_codes = torch.zeros(n, device=dev, dtype=torch.uint8)
        self.m_absmax = torch.zeros(nb, device=dev, dtype=torch.float32)
        self.v_absmax = torch.zeros(nb, device=dev, dtype=torch.float32)

    # -- (de)quantisation, torch reference -------------------------------------
    def _blocks(self, x):
        n = x.numel()
        pad = (-n) % self.BLOCK
        return torch.nn.functional.pad(x, (0, pad)).view(-1, self.BLOCK), n

    def dequant(self):
        mb, n = self._blocks(self.m_codes.float())
        vb, _ = self._blocks(self.v_codes.float())
        m = torch.sign(mb) * (mb.abs() / 127.0) ** 2 * self.m_absmax[:, None]
        v = (vb / 255.0) ** 4 * self.v_absmax[:, None]
        return m.reshape(-1)[:n], v.reshape(-1)[:n]

    def _quant(self, m, v):
        mb, n = self._blocks(m)
        vb, _ = self._blocks(v.clamp_min(0))
        am = mb.abs().amax(1)
        av = vb.amax(1)
        im = torch.where(am > 0, 1.0 / am, torch.zeros_like(am))[:, None]
        iv = torch.where(av > 0, 1.0 / av, torch.zeros_like(av))[:, None]
        mc = torch.round(127.0 * (mb.abs() * im).clamp(max=1).sqrt()) * torch.sign(mb)
        vc = torch.round(255.0 * (vb * iv).clamp(max=1).sqrt().sqrt())
        self.m_codes.copy_(mc.reshape(-1)[:n].to(torch.int8))
        self.v_codes.copy_(vc.reshape(-1)[:n].to(torch.uint8))
        self.m_absmax.copy_(am)
        self.v_absmax.copy_(av)

    def step(self, lr: float | None = None, use_clip: bool = False):
        if lr is not None:
            self.lr = lr
        self.step_count += 1
        b1, b2 = self.betas
        bc1 = 1.0 - b1 ** self.step_count
        bc2 = 1.0 - b2 ** self.step_count
        if self.native:
            mb = self.model_bf16  # as FlatAdamW.step: the kernel writes a bf16 copy only
            copy_after = mb is not None and mb.dtype != torch.bfloat16 and mb.data_ptr() != self.master.data_ptr()
            if mb is not None and mb.dtype != torch.bfloat16:
                mb = None
            _lib.call("kca_adamw8bit", self.master.data_ptr(), self.grad.data_ptr(), self.m_codes.data_ptr(),
                      self.m_absmax.data_ptr(), self.v_codes.data_ptr(), self.v_absmax.data_ptr(),
                      _lib.ptr(mb), self.master.numel(), _lib.ptr(self.wd_mask), float(self.lr),
                      float(b1), float(b2), float(self.eps), float(self.weight_decay), float(bc1), float(bc2),
                      self._coef.data_ptr() if use_clip else None,
                      self._skip.data_ptr() if use_clip else None, _lib.stream())
            if copy_after:
                self.model_bf16.copy_(self.master)
            return
        if use_clip and bool(self._skip.item()):
            return
        g = self.grad * (self._coef if use_clip else 1.0)
        m, v = self.dequant()
        m = b1 * m + (1 - b1) * g
        v = b2 * v + (1 - b2) * g * g
        denom = v.sqrt() / math.sqrt(bc2) + self.eps
        if self.weight_decay:
            if self.wd_mask is None:
                self.master.mul_(1 - self.lr * self.weight_decay)
            else:
                mk = self.wd_mask.to(self.master.device).bool().repeat_interleave(64)[: self.master.numel()]
                self.master.mul_(torch.where(mk, 1 - self.lr * self.weight_decay, 1.0))
        self.master.add_(-self.lr / bc1 * m / denom)
        self._quant(m, v)
        if self.model_bf16 is not None:
            self.model_bf16.copy_(self.master)

    def state_dict(self):
        return {"m_codes": self.m_codes, "v_codes": self.v_codes, "m_absmax": self.m_absmax,
                "v_absmax": self.v_absmax, "step": self.step_count, "lr": self.lr, "betas": list(self.betas),
                "eps": self.eps, "weight_decay": self.weight_decay, "bits": 8}

    def load_state_dict(self, sd):
        for k in ("m_codes", "v_codes", "m_absmax", "v_absmax"):
            getattr(self, k).copy_(sd[k])
        self.step_count = int(sd["step"])
        self.lr = sd.get("lr", self.lr)


class HostOffloadAdamW(FlatAdamW):
    """ZeRO-Offload style optimizer (N2 + PAR-3's ``offload_optimizer: cpu``,
    finetuner-workflow/finetuner/ds_config.json:35-37): fp32 master, exp_avg
    and exp_avg_sq of this rank's shard live in pinned HOST memory and are
    updated by the AVX-512/AVX2 host AdamW (csrc/cpu/adamw_host.cpp, OpenMP).

    Per step: the grad-norm clip coefficient is computed on the device (no extra
    traffic), the fp32 grad shard streams D2H in chunks on a copy stream while
    the host updates the previous chunk, and the bf16 result streams back H2D
    into the device parameters. Used only when the optimizer state would not
    fit in HBM (288 GB holds it for every model the
    reference trains on one node), or when forced for testing.
    """

    CHUNK = 1 << 24  # elements per D2H / host-update / H2D pipeline stage (64 MB fp32)

    def __init__(self, master: torch.Tensor, lr: float = 1e-3, betas=(0.9, 0.999), eps: float = 1e-8,
                 weight_decay: float = 0.0, wd_mask: torch.Tensor | None = None,
                 model_bf16: torch.Tensor | None = None, grad: torch.Tensor | None = None):
        dev = master.device
        pin = dev.type == "cuda"
        host_master = torch.empty(master.numel(), dtype=torch.float32, pin_memory=pin)
        host_master.copy_(master)
        super().__init__(host_master, lr, betas, eps, weight_decay, None, model_bf16, grad)
        # the base class put grad / clip scalars on the master's (host) device: keep
        # the grad where the engine accumulates it and the clip math on that device
        self.grad = grad if grad is not None else torch.zeros(master.numel(), device=dev)
        self.device = dev
        self._coef = torch.ones(1, device=dev, dtype=torch.float32)
        self._sumsq = torch.zeros(1, device=dev, dtype=torch.float32)
        self._norm = torch.zeros(1, device=dev, dtype=torch.float32)
        self._skip = torch.zeros(1, device=dev, dtype=torch.int32)
        self._ws = torch.empty(1024, device=dev, dtype=torch.float32)
        self.native = dev.type == "cuda"
        self.exp_avg = torch.zeros(master.numel(), dtype=torch.float32, pin_memory=pin)
        self.exp_avg_sq = torch.zeros(master.numel(), dtype=torch.float32, pin_memory=pin)
        self.wd_mask_host = wd_mask.cpu() if wd_mask is not None else None
        n = master.numel()
        c = min(self.CHUNK, n)
        self._g_host = [torch.empty(c, dtype=torch.float32, pin_memory=pin) for _ in range(2)]
        self._b_host = [torch.empty(c, dtype=torch.bfloat16, pin_memory=pin) for _ in range(2)]
        self._scal_host = torch.empty(2, dtype=torch.float32, pin_memory=pin)
        self._copy = torch.cuda.Stream(device=dev) if pin else None

    def step(self, lr: float | None = None, use_clip: bool = False):
        from ..io import native
        lib = native.load()
        if lr is not None:
            self.lr = lr
        self.step_count += 1
        b1, b2 = self.betas
        bc1 = 1.0 - b1 ** self.step_count
        bc2 = 1.0 - b2 ** self.step_count
        if use_clip:
            if bool(self._skip.item()):
                return
            gs = float(self._coef.item())
        else:
            gs = 1.0
        n = self.master.numel()
        mask = self.wd_mask_host
        cuda = self.device.type == "cuda"
        if cuda:
            cur = torch.cuda.current_stream(self.device)
            self._copy.wait_stream(cur)
        chunks = [(lo, min(n, lo + self.CHUNK)) for lo in range(0, n, self.CHUNK)]
        ev_in = [None, None]

        def fetch(i):
            lo, hi = chunks[i]
            buf = self._g_host[i & 1][: hi - lo]
            if cuda:
                with torch.cuda.stream(self._copy):
                    buf.copy_(self.grad[lo:hi], non_blocking=True)
                    ev_in[i & 1] = torch.cuda.Event()
                    ev_in[i & 1].record(self._copy)
            else:
                buf.copy_(self.grad[lo:hi])
            return buf

        pending = fetch(0) if chunks else None
        for i, (lo, hi) in enumerate(chunks):
            g = pending
            if cuda:
                ev_in[i & 1].synchronize()
            if i + 1 < len(chunks):
                pending = fetch(i + 1)
            pb = self._b_host[i & 1][: hi - lo]
            mk = mask[lo // 64:(hi + 63) // 64] if mask is not None else None
            lib.kca_host_adamw(self.master[lo:hi].data_ptr(), g.data_ptr(), self.exp_avg[lo:hi].data_ptr(),
                               self.exp_avg_sq[lo:hi].data_ptr(), pb.data_ptr(),
                               mk.data_ptr() if mk is not None else None, hi - lo, float(self.lr), float(b1),
                               float(b2), float(self.eps), float(self.weight_decay), float(bc1), float(bc2),
                               float(gs), 0)
            if self.model_bf16 is not None:
                if self.model_bf16.dtype != torch.bfloat16:  # fp32 model (CPU runs): exact copy
                    self.model_bf16[lo:hi].copy_(self.master[lo:hi])
                elif cuda:
                    self.model_bf16[lo:hi].copy_(pb, non_blocking=True)
                    # the host buffer is reused two chunks later: fence its upload
                    torch.cuda.current_stream(self.device).synchronize()
                else:
                    self.model_bf16[lo:hi].copy_(pb)


# ----------------------------------------------------------------- schedules
def lr_at(step: int, base_lr: float, total_steps: int, warmup_steps: int, kind: str = "linear",
          min_lr: float = 0.0) -> float:
    """HF-style schedules: warmup then linear / cosine / constant decay.

    ``kind='warmup'`` reproduces DeepSpeed WarmupLR (ds_config.json:19-26):
    linear warmup to ``base_lr`` then constant.
    """
    if warmup_steps > 0 and step < warmup_steps:
        return base_lr * float(step) / float(max(1, warmup_steps))
    if kind in ("constant", "warmup", "constant_with_warmup"):
        return base_lr
    progress = float(step - warmup_steps) / float(max(1, total_steps - warmup_steps))
    progress = min(max(progress, 0.0), 1.0)
    if kind == "cosine":
        return min_lr + (base_lr - min_lr) * 0.5 * (1.0 + math.cos(math.pi * progress))
    return max(0.0, base_lr * (1.0 - progress))


class DynamicLossScaler:
    """fp16 dynamic loss scale (ds_config.json:2-9: initial 2^16, window 1000,
    hysteresis 2, min 1)."""

    def __init__(self, init_scale: float = 2.0 ** 16, window: int = 1000, hysteresis: int = 2,
                 min_scale: float = 1.0, enabled: bool = True):
        self.scale = init_scale if enabled else 1.0
        self.window = window
        self.hysteresis = hysteresis
        self._hyst = hysteresis
        self.min_scale = min_scale
        self.enabled = enabled
        self._good = 0

    def update(self, overflow: bool):
        if not self.enabled:
            return
        if overflow:
            self._hyst -= 1
            if self._hyst <= 0:
                self.scale = max(self.min_scale, self.scale / 2.0)
                self._hyst = self.hysteresis
            self._good = 0
        else:
            self._good += 1
            if self._good % self.window == 0:
                self.scale *= 2.0
