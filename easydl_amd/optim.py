"""Optimizers over :class:`~easydl_amd.parallel.flat.FlatParams`.

``FlatAdamW`` keeps fp32 master weights and fp32 moments as flat buffers next
to the bf16 model weights (16 B/param of state: Llama-3-8B = 128 GB, which
fits a single 288 GB MI355X with room for activations — SURVEY.md §2.9), and
performs the whole update with one fused kernel launch per group after one
grad-norm/clip reduction whose result never leaves the device.
"""
from __future__ import annotations

import math

import torch

from easydl_amd.ops.optim import adamw_flat_, grad_clip_scale, sgd_flat_
from easydl_amd.parallel.flat import FlatParams
from easydl_amd.utils import vram


class LRSchedule:
    """Linear warmup then cosine decay to ``min_ratio * lr``."""

    def __init__(self, lr: float, warmup: int = 0, total: int = 0, min_ratio: float = 0.1):
        self.lr, self.warmup, self.total, self.min_ratio = lr, warmup, total, min_ratio

    def __call__(self, step: int) -> float:
        if self.warmup and step <= self.warmup:
            return self.lr * step / self.warmup
        if not self.total or step >= self.total:
            return self.lr if not self.total else self.lr * self.min_ratio
        p = (step - self.warmup) / max(1, self.total - self.warmup)
        return self.lr * (self.min_ratio + (1 - self.min_ratio) * 0.5 * (1 + math.cos(math.pi * p)))

    def state_dict(self):
        return dict(lr=self.lr, warmup=self.warmup, total=self.total, min_ratio=self.min_ratio)


def rehome_state(state: list, adopted, can_continue=lambda: True) -> int:
    """Optimizer-state tensors on adopted memory -> own copies (see FlatParams.rehome)."""
    n = 0
    with torch.no_grad():
        for st in state:
            for k, t in list(st.items()):
                if isinstance(t, torch.Tensor) and adopted(t) and can_continue():
                    st[k] = t.clone()
                    n += 1
    return n


def _zeros(name: str, g, dtype=torch.float32) -> torch.Tensor:
    """Optimizer state of flat group ``g``: a buffer handed over by the previous worker on
    this GPU (utils/vram.py, its values kept for an HBM resume), or a new zeroed one."""
    t = vram.take(name, g.numel, dtype, g.data.device, keep=True)
    return torch.zeros(g.numel, dtype=dtype, device=g.data.device) if t is None else t


class FlatAdamW:
    """``moment_dtype``: fp32 (default) or bf16 moments -- 8 instead of 12 B/param of state,
    stochastically rounded with deterministic random bits (ops/optim.py bf16_stochastic), so
    snapshot + resume stays bit-exact; chosen when fp32 moments would not fit two full
    in-memory snapshot slots in the rank's host DRAM (ElasticTrainer, ``moment_dtype="auto"``)."""

    def __init__(self, flat: FlatParams, lr: float = 3e-4, betas=(0.9, 0.95), eps: float = 1e-8,
                 weight_decay: float | None = None, max_grad_norm: float = 1.0, schedule: LRSchedule | None = None,
                 moment_dtype: torch.dtype = torch.float32):
        if moment_dtype not in (torch.float32, torch.bfloat16):
            raise ValueError(f"moment_dtype must be float32 or bfloat16, got {moment_dtype}")
        self.moment_dtype = moment_dtype
        self.flat = flat
        self.lr = lr
        self.beta1, self.beta2 = betas
        self.eps = eps
        self.max_grad_norm = max_grad_norm
        self.schedule = schedule
        self.step_count = 0
        # step at which the moments (m, v) last started from zero: bias correction counts
        # from here (a lean snapshot restores the master weights only, ckpt/manager.py)
        self.moment_origin = 0
        self.last_stats = None  # device tensor [coef, norm, nonfinite]
        # model parallelism: per-group sum-of-squares weights + group all-reduce
        self.norm_weights = None
        self.norm_reduce = None
        self.state = []
        for g in flat.groups:
            if weight_decay is not None and g.name.startswith("decay"):
                g.weight_decay = weight_decay
            has16 = g.data.dtype != torch.float32
            if has16:
                master = vram.take(f"opt/{g.name}/master", g.numel, torch.float32, g.data.device, keep=True)
                master = g.data.float() if master is None else master
            else:
                master = g.data
            self.state.append({"master": master, "m": _zeros(f"opt/{g.name}/m", g, moment_dtype),
                               "v": _zeros(f"opt/{g.name}/v", g, moment_dtype)})

    def current_lr(self) -> float:
        return self.schedule(self.step_count + 1) if self.schedule else self.lr

    @torch.no_grad()
    def set_moment_dtype(self, dtype: torch.dtype) -> bool:
        """Switch the moment buffers to ``dtype`` (the job's agreed choice, ElasticTrainer
        _agree_moment_dtype); values are converted.  Returns True if anything changed."""
        if dtype not in (torch.float32, torch.bfloat16):
            raise ValueError(f"moment_dtype must be float32 or bfloat16, got {dtype}")
        if dtype == self.moment_dtype:
            return False
        for st in self.state:
            st["m"] = st["m"].to(dtype)
            st["v"] = st["v"].to(dtype)
        self.moment_dtype = dtype
        return True

    @torch.no_grad()
    def reset_state(self) -> None:
        """Fresh-start optimizer state for the current weights: master = weights, zero moments
        (after :meth:`FlatParams.reinit_adopted`)."""
        for g, st in zip(self.flat.groups, self.state):
            if st["master"].data_ptr() != g.data.data_ptr():
                st["master"].copy_(g.data)
            st["m"].zero_()
            st["v"].zero_()
        self.step_count = 0
        self.moment_origin = 0

    supports_group_done = True

    @torch.no_grad()
    def step(self, pre_scale: float = 1.0, group_done=None) -> torch.Tensor:
        """Apply one update; ``pre_scale`` multiplies the (summed) gradients, e.g. 1/world.
        ``group_done(i)``: called after group i's update is enqueued; the groups then go last
        to first -- the order the next forward reads them (FlatParams lays parameters out in
        reverse registration order), so it can start on the first groups while the rest update
        (ElasticTrainer._opt_overlap)."""
        grads = [g.grad for g in self.flat.groups]
        stats = grad_clip_scale(grads, self.max_grad_norm, pre_scale, self.norm_weights, self.norm_reduce)
        self.step_count += 1
        lr = self.schedule(self.step_count) if self.schedule else self.lr
        order = range(len(self.state) - 1, -1, -1) if group_done is not None else range(len(self.state))
        for i in order:
            g, st = self.flat.groups[i], self.state[i]
            p16 = g.data if g.data.dtype != torch.float32 else None
            adamw_flat_(p16, st["master"], st["m"], st["v"], g.grad, lr=lr, beta1=self.beta1, beta2=self.beta2,
                        eps=self.eps, weight_decay=g.weight_decay, step=self.step_count - self.moment_origin,
                        dscale=stats)
            if group_done is not None:
                group_done(i)
        self.last_stats = stats
        return stats

    # -- checkpoint ------------------------------------------------------------
    def state_tensors(self) -> dict[str, torch.Tensor]:
        """Flat tensors that fully describe optimizer state (model data excluded)."""
        out = {}
        for g, st in zip(self.flat.groups, self.state):
            if st["master"].data_ptr() != g.data.data_ptr():
                out[f"opt.{g.name}.master"] = st["master"]
            out[f"opt.{g.name}.m"] = st["m"]
            out[f"opt.{g.name}.v"] = st["v"]
        return out

    def moment_names(self) -> set[str]:
        return {n for n in self.state_tensors() if n.endswith((".m", ".v"))}

    def scalars(self) -> dict:
        return {"step_count": self.step_count, "lr": self.lr, "moment_origin": self.moment_origin}

    def load_scalars(self, d: dict) -> None:
        self.step_count = int(d["step_count"])
        self.moment_origin = int(d.get("moment_origin", 0))


class FlatSGD:
    def __init__(self, flat: FlatParams, lr: float = 0.1, momentum: float = 0.9, weight_decay: float = 0.0,
                 max_grad_norm: float = 0.0, schedule: LRSchedule | None = None):
        self.flat = flat
        self.lr, self.momentum, self.max_grad_norm, self.schedule = lr, momentum, max_grad_norm, schedule
        self.norm_weights = None
        self.norm_reduce = None
        self.step_count = 0
        self.state = []
        for g in flat.groups:
            if g.name.startswith("decay"):
                g.weight_decay = weight_decay
            has16 = g.data.dtype != torch.float32
            self.state.append({
                "master": g.data.float() if has16 else g.data,
                "mom": _zeros(f"opt/{g.name}/mom", g) if momentum else None,
            })

    @torch.no_grad()
    def reset_state(self) -> None:
        """See :meth:`FlatAdamW.reset_state`."""
        for g, st in zip(self.flat.groups, self.state):
            if st["master"].data_ptr() != g.data.data_ptr():
                st["master"].copy_(g.data)
            if st["mom"] is not None:
                st["mom"].zero_()
        self.step_count = 0

    @torch.no_grad()
    def step(self, pre_scale: float = 1.0):
        grads = [g.grad for g in self.flat.groups]
        stats = grad_clip_scale(grads, self.max_grad_norm, pre_scale, self.norm_weights, self.norm_reduce)
        self.step_count += 1
        lr = self.schedule(self.step_count) if self.schedule else self.lr
        for g, st in zip(self.flat.groups, self.state):
            p16 = g.data if g.data.dtype != torch.float32 else None
            sgd_flat_(p16, st["master"], st["mom"], g.grad, lr=lr, momentum=self.momentum,
                      weight_decay=g.weight_decay, dscale=stats)
        return stats

    def state_tensors(self):
        out = {}
        for g, st in zip(self.flat.groups, self.state):
            if st["master"].data_ptr() != g.data.data_ptr():
                out[f"opt.{g.name}.master"] = st["master"]
            if st["mom"] is not None:
                out[f"opt.{g.name}.mom"] = st["mom"]
        return out

    def moment_names(self) -> set[str]:
        return {n for n in self.state_tensors() if n.endswith(".mom")}

    def scalars(self):
        return {"step_count": self.step_count, "lr": self.lr}

    def load_scalars(self, d):
        self.step_count = int(d["step_count"])
