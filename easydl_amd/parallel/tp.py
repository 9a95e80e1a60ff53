"""Megatron-style tensor parallelism for the Llama family (BASELINE.json config 5:
Llama-3 70B, TP=8 over xGMI).

Per TP rank of ``tp`` ranks:
* attention: the fused QKV weight holds H/tp query heads and KV/tp key/value
  heads (70B: 8 q-heads + 1 kv-head per GPU), the output projection holds the
  matching H/tp*D input columns -> its partial output is all-reduced;
* MLP: the fused [gate | up] weight holds F/tp rows of each half (so SwiGLU
  stays local), the down projection the matching F/tp columns -> all-reduce;
* embedding and LM head are vocab-parallel (V/tp rows each); the cross
  entropy combines max / sum-exp / target logit with three tiny all-reduces
  and never materialises the full-vocab logits;
* norms are replicated (their inputs are replicated after each all-reduce, so
  their gradients are identical on every TP rank — no reduction needed).

The conjugate operators ``copy_to_tp`` (identity fwd / all-reduce bwd) and
``reduce_from_tp`` (all-reduce fwd / identity bwd) carry the two all-reduces
per block in each direction: [T, d] bf16 = 64 MiB at 4k tokens x d=8192 for
70B — large messages that keep all 7 xGMI links of a node busy.
Sequence parallelism (P4) swaps each all-reduce for reduce-scatter +
all-gather over the token dimension (``sequence_parallel=True``).

Without SP the collectives overlap compute (``EDL_TP_OVERLAP``, default on): a
row-parallel GEMM runs in row chunks and each chunk's all-reduce starts on the
communicator's stream while the next chunk multiplies; a column-parallel GEMM's
input-gradient all-reduce starts as soon as dX exists and runs under the
weight-gradient GEMMs (``fused.linear`` / ``fused.swiglu_mlp`` hooks).  With SP,
the column-parallel weight gradients run on the side stream so each input
gradient's reduce-scatter overlaps them.
"""
from __future__ import annotations

import os

import torch
import torch.distributed as dist
import torch.nn as nn
import torch.utils.checkpoint as _ckpt

from easydl_amd.models.llama import Llama, LlamaBlock, LlamaConfig, _param
from easydl_amd.ops import fused, norms


class TPGroup:
    """TP ranks of one model replica (wraps an epoch Communicator).

    Under the elastic trainer the group outlives epochs: the model is built
    once against it and :meth:`rebind` swaps in each new epoch's TP
    communicator (same size; the rank may change, with the state re-synced).
    """

    def __init__(self, comm=None, sequence_parallel: bool = False, size: int | None = None, rank: int = 0):
        self.comm = comm
        self.rank = comm.rank if comm is not None else rank
        self.size = comm.world_size if comm is not None else int(size or 1)
        self.sequence_parallel = sequence_parallel

    def rebind(self, comm) -> None:
        if comm.world_size != self.size:
            raise ValueError(f"TP size is fixed at {self.size}, got a group of {comm.world_size}")
        self.comm, self.rank = comm, comm.rank

    def all_reduce(self, x: torch.Tensor) -> torch.Tensor:
        if self.size == 1:
            return x
        x = x.contiguous()
        self.comm.all_reduce(x)
        return x

    def all_reduce_start(self, x: torch.Tensor):
        """Start an in-place SUM of ``x`` (contiguous) on the communicator's stream;
        returns ``finish()``, which orders the compute stream after it and returns x.
        The overlap hooks of ``fused.linear`` / ``fused.swiglu_mlp`` use it."""
        work = self.comm.all_reduce_async(x)

        def finish():
            self.comm.wait_work(work)
            return x
        return finish

    def all_reduce_max(self, x: torch.Tensor) -> torch.Tensor:
        if self.size == 1:
            return x
        x = x.contiguous()
        self.comm.all_reduce(x, dist.ReduceOp.MAX)
        return x

    def all_gather_rows(self, x: torch.Tensor) -> torch.Tensor:
        if self.size == 1:
            return x
        out = torch.empty(x.shape[0] * self.size, *x.shape[1:], dtype=x.dtype, device=x.device)
        self.comm.all_gather_into(out, x.contiguous())
        return out

    def reduce_scatter_rows(self, x: torch.Tensor) -> torch.Tensor:
        if self.size == 1:
            return x
        out = torch.empty(x.shape[0] // self.size, *x.shape[1:], dtype=x.dtype, device=x.device)
        self.comm.reduce_scatter_into(out, x.contiguous())
        return out


class _CopyToTP(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, g):
        ctx.g = g
        return x

    @staticmethod
    def backward(ctx, dy):
        return ctx.g.all_reduce(dy.clone()), None


class _ReduceFromTP(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, g):
        return g.all_reduce(x.clone())

    @staticmethod
    def backward(ctx, dy):
        return dy, None


class _GatherFromSP(torch.autograd.Function):
    """SP: [T/tp, d] -> [T, d] (all-gather); backward reduce-scatter."""

    @staticmethod
    def forward(ctx, x, g):
        ctx.g = g
        return g.all_gather_rows(x)

    @staticmethod
    def backward(ctx, dy):
        return ctx.g.reduce_scatter_rows(dy), None


class _ScatterToSP(torch.autograd.Function):
    """SP: partial [T, d] -> reduce-scatter -> [T/tp, d]; backward all-gather."""

    @staticmethod
    def forward(ctx, x, g):
        ctx.g = g
        return g.reduce_scatter_rows(x)

    @staticmethod
    def backward(ctx, dy):
        return ctx.g.all_gather_rows(dy), None


def copy_to_tp(x, g: TPGroup):
    return _CopyToTP.apply(x, g) if g.size > 1 else x


def gather_from_sp(x, g: TPGroup):
    return _GatherFromSP.apply(x, g) if g.size > 1 else x


def scatter_to_sp(x, g: TPGroup):
    return _ScatterToSP.apply(x, g) if g.size > 1 else x


def reduce_from_tp(x, g: TPGroup):
    return _ReduceFromTP.apply(x, g) if g.size > 1 else x


class _VocabParallelXent(torch.autograd.Function):
    @staticmethod
    def forward(ctx, logits, labels, vstart, g, ignore_index):
        x = logits.float()
        m = x.max(dim=-1).values
        m = g.all_reduce_max(m)
        e = torch.exp(x - m[:, None])
        s = g.all_reduce(e.sum(-1))
        local = (labels >= vstart) & (labels < vstart + x.shape[-1])
        idx = (labels - vstart).clamp(0, x.shape[-1] - 1)
        tgt = torch.where(local, x.gather(1, idx[:, None])[:, 0], torch.zeros_like(m))
        tgt = g.all_reduce(tgt)
        valid = labels != ignore_index
        loss_rows = torch.where(valid, torch.log(s) + m - tgt, torch.zeros_like(m))
        n = valid.sum().clamp_min(1).float()
        p = e / s[:, None]
        ctx.save_for_backward(p, idx, local & valid, valid, n)
        ctx.dtype = logits.dtype
        return loss_rows.sum() / n

    @staticmethod
    def backward(ctx, dl):
        p, idx, hit, valid, n = ctx.saved_tensors
        grad = p * valid[:, None].float()
        grad[hit.nonzero()[:, 0], idx[hit]] -= 1.0
        return (grad * (dl / n)).to(ctx.dtype), None, None, None, None


class _VocabParallelXentHip(torch.autograd.Function):
    """GPU form (csrc/kernels/fused.hip ``edl_xent_vp``): one pass over the bf16 local
    logits gives per-row (max, sum-exp, target logit); the ranks combine them with one
    MAX all-reduce of [T] fp32 and one SUM all-reduce of [T, 2] fp32; the backward
    rewrites the logits in place with their gradient.  No fp32 [T, V/tp] tensor is
    ever materialised (the eager form held x, e and p in fp32)."""

    @staticmethod
    def forward(ctx, logits, labels, vstart, g, ignore_index):
        from easydl_amd import _native
        k = _native.kernels()
        logits = logits.contiguous()
        rows, V = logits.shape
        labels = labels.contiguous().to(torch.int64)
        st = torch.empty(rows, 3, dtype=torch.float32, device=logits.device)
        k.check("edl_xent_vp", logits.data_ptr(), labels.data_ptr(), st.data_ptr(), rows, V, vstart, ignore_index,
                0, None, _native.stream_of(logits))
        m_loc = st[:, 0]
        M = g.all_reduce_max(m_loc.clone())
        sums = torch.stack([st[:, 1] * torch.exp(m_loc - M), st[:, 2]], 1)
        sums = g.all_reduce(sums)
        S, tgt = sums[:, 0], sums[:, 1]
        valid = labels != ignore_index
        n = valid.sum().clamp_min(1).float()
        loss = torch.where(valid, torch.log(S) + M - tgt, torch.zeros_like(M)).sum() / n
        if ctx.needs_input_grad[0]:
            ctx.save_for_backward(logits, labels, torch.stack([M, S], 1).contiguous(), n)
            ctx.vstart, ctx.ignore_index = vstart, ignore_index
        return loss

    @staticmethod
    def backward(ctx, dl):
        from easydl_amd import _native
        if getattr(ctx, "consumed", False):
            raise RuntimeError("vocab-parallel cross_entropy: backward ran twice (logits consumed in place)")
        ctx.consumed = True
        logits, labels, ms, n = ctx.saved_tensors
        rows, V = logits.shape
        scale = (dl.float() / n).reshape(1).contiguous()
        _native.kernels().check("edl_xent_vp", logits.data_ptr(), labels.data_ptr(), ms.data_ptr(), rows, V,
                                ctx.vstart, ctx.ignore_index, 1, scale.data_ptr(), _native.stream_of(logits))
        return logits, None, None, None, None


def vocab_parallel_cross_entropy(logits_local, labels, vstart: int, g: TPGroup, ignore_index: int = -100):
    if logits_local.is_cuda and logits_local.dtype == torch.bfloat16 and logits_local.shape[-1] % 8 == 0:
        return _VocabParallelXentHip.apply(logits_local.reshape(-1, logits_local.shape[-1]), labels.reshape(-1),
                                           vstart, g, ignore_index)
    return _VocabParallelXent.apply(logits_local, labels.reshape(-1), vstart, g, ignore_index)


class LlamaTP(nn.Module):
    """One TP rank of a Llama model (parameter names match :class:`Llama`)."""

    def __init__(self, cfg: LlamaConfig, g: TPGroup, device=None, dtype=torch.bfloat16):
        super().__init__()
        tp = g.size
        if cfg.n_heads % tp or cfg.n_kv_heads % tp or cfg.ffn_dim % tp or cfg.vocab_size % tp:
            raise ValueError(f"config not divisible by tp={tp}")
        self.cfg, self.g = cfg, g
        self.vshard = cfg.vocab_size // tp
        on = os.environ.get("EDL_TP_OVERLAP", "1") != "0"
        self.overlap = tp > 1 and not g.sequence_parallel and on
        self.sp_overlap = tp > 1 and g.sequence_parallel and on
        d = cfg.dim
        self.embed = _param((self.vshard, d), cfg.init_std, device, dtype)
        self.layers = nn.ModuleList()
        for _ in range(cfg.n_layers):
            blk = LlamaBlock(cfg, device, dtype, n_heads=cfg.n_heads // tp, n_kv_heads=cfg.n_kv_heads // tp,
                             ffn_dim=cfg.ffn_dim // tp)
            if g.sequence_parallel:
                # Megatron-SP: the residual stream and norms live on a 1/tp token shard;
                # all-gather before the column-parallel GEMMs, reduce-scatter after the
                # row-parallel ones (same bytes as the all-reduce, 1/tp the activations)
                blk.tp_reduce = lambda x, _g=g: scatter_to_sp(x, _g)
                blk.tp_copy = lambda x, _g=g: gather_from_sp(x, _g)
                # the reduce-scatter of each column-parallel input gradient runs beside that
                # GEMM's weight gradient (side stream) instead of after it
                blk.tp_wgrad_side = self.sp_overlap
            elif self.overlap:
                # the two all-reduces per block run beside GEMMs: the row-parallel outputs
                # chunk by chunk behind their own GEMM, the column-parallel input gradients
                # under the weight-gradient GEMMs (fused.linear / swiglu_mlp hooks)
                blk.tp_out_reduce = blk.tp_dx_reduce = g.all_reduce_start
            else:
                blk.tp_reduce = lambda x, _g=g: reduce_from_tp(x, _g)
                blk.tp_copy = lambda x, _g=g: copy_to_tp(x, _g)
            self.layers.append(blk)
        self.norm = _param((d,), 0, device, dtype)
        self.lm_head = _param((self.vshard, d), cfg.init_std, device, dtype)
        self._rope = {}
        # norms are replicated on every TP rank (identical values and gradients):
        # the grad-norm counts them once (ElasticTrainer / FlatAdamW weights)
        for n, p in self.named_parameters():
            if p.ndim < 2:
                p._tp_replicated = True

    rope = Llama.rope

    def sync_sp_grads(self, flat=None) -> None:
        """Sequence parallelism: each TP rank's norm weights saw only its token shard,
        so their gradients are partial — sum them over the TP group (after backward,
        before clipping).  ``flat``: a FlatParams whose groups hold these parameters
        (one all-reduce per group) — else per parameter."""
        if not self.g.sequence_parallel or self.g.size == 1:
            return
        if flat is not None:
            for grp in flat.groups:
                if grp.slots and all(getattr(sl.param, "_tp_replicated", False) for sl in grp.slots):
                    self.g.all_reduce(grp.grad)
            return
        for p in self.parameters():
            if getattr(p, "_tp_replicated", False) and p.grad is not None:
                p.grad.copy_(self.g.all_reduce(p.grad))

    @property
    def vstart(self) -> int:  # follows the group's current rank (elastic re-ranking)
        return self.g.rank * self.vshard

    def forward(self, ids, labels=None):
        B, S = ids.shape
        cos, sin = self.rope(S, ids.device)
        flat = ids.reshape(-1)
        local = (flat >= self.vstart) & (flat < self.vstart + self.vshard)
        x = fused.embedding((flat - self.vstart).clamp(0, self.vshard - 1), self.embed)
        x = x * local[:, None].to(x.dtype)
        sp = self.g.sequence_parallel and self.g.size > 1
        if sp and flat.numel() % self.g.size:
            raise ValueError(f"sequence parallelism needs B*S ({flat.numel()}) divisible by tp={self.g.size}")
        x = scatter_to_sp(x, self.g) if sp else reduce_from_tp(x, self.g)
        resid, delta = x, None
        for layer in self.layers:
            if self.cfg.recompute and self.training:
                # activation recompute (the 80-layer 70B shard at 8k tokens: profiles/r04_tp_dryrun_*);
                # the re-run forward repeats the block's TP collectives, as in Megatron
                resid, delta = _ckpt.checkpoint(layer, resid, delta, B, S, cos, sin, use_reentrant=False)
            else:
                resid, delta = layer(resid, delta, B, S, cos, sin)
        n, _ = norms.add_rmsnorm(delta, resid, self.norm, self.cfg.norm_eps)
        if self.overlap:
            logits = fused.linear(n, self.lm_head, dx_reduce=self.g.all_reduce_start)
        else:
            n = gather_from_sp(n, self.g) if sp else copy_to_tp(n, self.g)
            logits = fused.linear(n, self.lm_head, wgrad_side=self.sp_overlap)
        if labels is None:
            return logits
        return vocab_parallel_cross_entropy(logits, labels, self.vstart, self.g)


def shard_state_dict(full: dict[str, torch.Tensor], cfg: LlamaConfig, rank: int, tp: int) -> dict[str, torch.Tensor]:
    """Slice a dense :class:`Llama` state dict into TP rank ``rank`` of ``tp``."""
    H, KV, D, F = cfg.n_heads, cfg.n_kv_heads, cfg.head_dim, cfg.ffn_dim
    hs, ks, fs, vs = H // tp, KV // tp, F // tp, cfg.vocab_size // tp
    out = {}
    for name, w in full.items():
        if name.endswith("wqkv"):
            q = w[:H * D].view(H, D, -1)[rank * hs:(rank + 1) * hs].reshape(hs * D, -1)
            k = w[H * D:(H + KV) * D].view(KV, D, -1)[rank * ks:(rank + 1) * ks].reshape(ks * D, -1)
            v = w[(H + KV) * D:].view(KV, D, -1)[rank * ks:(rank + 1) * ks].reshape(ks * D, -1)
            out[name] = torch.cat([q, k, v])
        elif name.endswith("wo"):
            out[name] = w[:, rank * hs * D:(rank + 1) * hs * D]
        elif name.endswith("w_gu"):
            out[name] = torch.cat([w[rank * fs:(rank + 1) * fs], w[F + rank * fs:F + (rank + 1) * fs]])
        elif name.endswith("w_down"):
            out[name] = w[:, rank * fs:(rank + 1) * fs]
        elif name in ("embed", "lm_head"):
            out[name] = w[rank * vs:(rank + 1) * vs]
        else:
            out[name] = w
    return {k: v.contiguous() for k, v in out.items()}
