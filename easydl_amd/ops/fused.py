"""Fused transformer ops: SwiGLU, RoPE+QKV split, softmax cross-entropy,
direct-gradient Linear and Embedding.

HIP kernels live in ``csrc/kernels/fused.hip``; GEMMs go to hipBLASLt through
``torch.mm`` (plain library GEMMs) with the weight gradient written straight
into the flat gradient buffer (see :mod:`easydl_amd.ops.gradsink`).
"""
from __future__ import annotations

import math
import os
import weakref

import torch
import torch.nn.functional as F

from easydl_amd import _native
from easydl_amd.ops import gradsink


# ----------------------------------------------------------------------------
# SwiGLU over the packed [gate | up] projection
# ----------------------------------------------------------------------------
def swiglu_ref(gu: torch.Tensor) -> torch.Tensor:
    g, u = gu.float().chunk(2, dim=-1)
    return (F.silu(g) * u).to(gu.dtype)


class _SwiGLUFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, gu):
        k = _native.kernels()
        gu = gu.contiguous()
        F2 = gu.shape[-1]
        rows = gu.numel() // F2
        out = torch.empty(*gu.shape[:-1], F2 // 2, dtype=gu.dtype, device=gu.device)
        k.check("edl_swiglu_fwd", gu.data_ptr(), out.data_ptr(), rows, F2 // 2, _native.stream_of(gu))
        ctx.save_for_backward(gu)
        return out

    @staticmethod
    def backward(ctx, dout):
        k = _native.kernels()
        (gu,) = ctx.saved_tensors
        dout = dout.contiguous()
        F2 = gu.shape[-1]
        rows = gu.numel() // F2
        dgu = torch.empty_like(gu)
        k.check("edl_swiglu_bwd", dout.data_ptr(), gu.data_ptr(), dgu.data_ptr(), rows, F2 // 2,
                _native.stream_of(gu))
        return dgu


def swiglu(gu: torch.Tensor) -> torch.Tensor:
    if _native.use_hip(gu):
        if gu.dtype != torch.bfloat16:
            raise TypeError("swiglu kernel expects bf16")
        return _SwiGLUFn.apply(gu)
    return swiglu_ref(gu)


# ----------------------------------------------------------------------------
# Rotary embedding fused with the QKV split
# ----------------------------------------------------------------------------
def rope_tables(seq_len: int, head_dim: int, theta: float = 500000.0, device=None,
                scaling: dict | None = None):
    """cos/sin tables [S, D/2] fp32 (rotate-half convention, Llama-3 frequencies).

    ``scaling`` implements Llama-3.1 style frequency scaling when given
    (``factor``, ``low_freq_factor``, ``high_freq_factor``, ``original_max_position_embeddings``).
    """
    inv = 1.0 / (theta ** (torch.arange(0, head_dim, 2, dtype=torch.float64) / head_dim))
    if scaling:
        factor = scaling.get("factor", 8.0)
        lo = scaling.get("low_freq_factor", 1.0)
        hi = scaling.get("high_freq_factor", 4.0)
        old = scaling.get("original_max_position_embeddings", 8192)
        wavelen = 2 * math.pi / inv
        lo_wl, hi_wl = old / lo, old / hi
        smooth = (old / wavelen - lo) / (hi - lo)
        scaled = torch.where(wavelen > lo_wl, inv / factor, inv)
        mid = (wavelen <= lo_wl) & (wavelen >= hi_wl)
        inv = torch.where(mid, (1 - smooth) * inv / factor + smooth * inv, scaled)
    t = torch.arange(seq_len, dtype=torch.float64)
    fr = torch.outer(t, inv)
    return fr.cos().float().to(device), fr.sin().float().to(device)


def rope_qkv_ref(qkv, cos, sin, B, S, H, KV, D):
    """qkv [B*S, (H+2KV)*D] -> q [B,H,S,D], k [B,KV,S,D], v [B,KV,S,D] (fp32 math)."""
    x = qkv.float().view(B, S, H + 2 * KV, D)
    q, k, v = x[:, :, :H], x[:, :, H:H + KV], x[:, :, H + KV:]
    c = cos[:S].view(1, S, 1, D // 2)
    s = sin[:S].view(1, S, 1, D // 2)

    def rot(t):
        a, b = t[..., : D // 2], t[..., D // 2:]
        return torch.cat([a * c - b * s, b * c + a * s], dim=-1)

    dt = qkv.dtype
    return (rot(q).to(dt).transpose(1, 2), rot(k).to(dt).transpose(1, 2), v.to(dt).transpose(1, 2))


class _RopeQKVFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, qkv, cos, sin, B, S, H, KV, D):
        k_ = _native.kernels()
        qkv = qkv.contiguous()
        T = B * S
        q = torch.empty(B, S, H, D, dtype=qkv.dtype, device=qkv.device)
        k = torch.empty(B, S, KV, D, dtype=qkv.dtype, device=qkv.device)
        v = torch.empty(B, S, KV, D, dtype=qkv.dtype, device=qkv.device)
        k_.check("edl_rope_qkv_fwd", qkv.data_ptr(), q.data_ptr(), k.data_ptr(), v.data_ptr(), cos.data_ptr(),
                 sin.data_ptr(), T, S, H, KV, D, _native.stream_of(qkv))
        ctx.save_for_backward(cos, sin)
        ctx.dims = (B, S, H, KV, D)
        # [B,H,S,D] views of [B,S,H,D] memory: what flash attention consumes copy-free
        return q.transpose(1, 2), k.transpose(1, 2), v.transpose(1, 2)

    @staticmethod
    def backward(ctx, dq, dk, dv):
        k_ = _native.kernels()
        cos, sin = ctx.saved_tensors
        B, S, H, KV, D = ctx.dims
        dev = cos.device
        dt = (dq if dq is not None else dk if dk is not None else dv).dtype

        def bshd(t, heads):
            if t is None:
                return torch.zeros(B, S, heads, D, dtype=dt, device=dev)
            return t.transpose(1, 2).contiguous()

        dq_, dk_, dv_ = bshd(dq, H), bshd(dk, KV), bshd(dv, KV)
        dqkv = torch.empty(B * S, (H + 2 * KV) * D, dtype=dt, device=dev)
        k_.check("edl_rope_qkv_bwd", dq_.data_ptr(), dk_.data_ptr(), dv_.data_ptr(), dqkv.data_ptr(), cos.data_ptr(),
                 sin.data_ptr(), B * S, S, H, KV, D, _native.stream_of(dqkv))
        return dqkv, None, None, None, None, None, None, None


def rope_qkv(qkv, cos, sin, B, S, H, KV, D):
    if _native.use_hip(qkv):
        return _RopeQKVFn.apply(qkv, cos, sin, B, S, H, KV, D)
    return rope_qkv_ref(qkv, cos, sin, B, S, H, KV, D)


# ----------------------------------------------------------------------------
# Softmax cross-entropy (forward computes the gradient in place)
# ----------------------------------------------------------------------------
def cross_entropy_ref(logits, labels, ignore_index=-100):
    return F.cross_entropy(logits.float(), labels, ignore_index=ignore_index)


_XENT_LSE = os.environ.get("EDL_XENT_LSE", "1") != "0"


class _XentFn(torch.autograd.Function):
    """Mean token cross-entropy over bf16 logits.  The forward only reads the logits
    (loss and log-sum-exp per row); the backward writes the final gradient
    (exp(x - lse) - onehot) * dloss / n_valid in place into the logits buffer: one read +
    one write, instead of a write in the forward plus a separate scaling pass (-1.8 ms per
    16k x 128k micro-batch) and without re-reading the row for its statistics
    (EDL_XENT_LSE=0: the backward recomputes them)."""

    @staticmethod
    def forward(ctx, logits, labels, ignore_index):
        k = _native.kernels()
        if not logits.is_contiguous():
            logits = logits.contiguous()
        rows, V = logits.shape
        loss = torch.empty(rows, dtype=torch.float32, device=logits.device)
        lse = torch.empty(rows, dtype=torch.float32, device=logits.device) if _XENT_LSE else None
        labels = labels.contiguous().to(torch.int64)
        k.check("edl_xent_fwd_bwd", logits.data_ptr(), labels.data_ptr(), loss.data_ptr(), rows, V, ignore_index,
                0, None, _native.ptr(lse), _native.stream_of(logits))
        nvalid = (labels != ignore_index).sum().clamp_min(1).float()
        out = loss.sum() / nvalid
        if ctx.needs_input_grad[0]:
            ctx.save_for_backward(logits, labels, nvalid, loss, lse)
            ctx.ignore_index = ignore_index
        return out

    @staticmethod
    def backward(ctx, dloss):
        k = _native.kernels()
        if getattr(ctx, "consumed", False):
            # the first backward turned the saved logits into their gradient in place
            raise RuntimeError("fused cross_entropy: backward ran twice (retain_graph is not supported: "
                               "the logits buffer is consumed by its gradient)")
        ctx.consumed = True
        logits, labels, nvalid, loss, lse = ctx.saved_tensors
        rows, V = logits.shape
        scale = (dloss.float() / nvalid).reshape(1).contiguous()
        # NOTE: the saved logits buffer becomes its own gradient (no second V x rows buffer)
        if lse is not None:
            k.check("edl_xent_grad_lse", logits.data_ptr(), labels.data_ptr(), lse.data_ptr(), rows, V,
                    ctx.ignore_index, scale.data_ptr(), _native.stream_of(logits))
        else:
            k.check("edl_xent_fwd_bwd", logits.data_ptr(), labels.data_ptr(), loss.data_ptr(), rows, V,
                    ctx.ignore_index, 1, scale.data_ptr(), None, _native.stream_of(logits))
        return logits, None, None


def cross_entropy(logits, labels, ignore_index: int = -100):
    """Mean token cross-entropy. On GPU the bf16 logits buffer is consumed (overwritten by its gradient)."""
    if _native.use_hip(logits) and logits.dtype == torch.bfloat16 and logits.shape[-1] % 8 == 0:
        return _XentFn.apply(logits.view(-1, logits.shape[-1]), labels.reshape(-1), ignore_index)
    return cross_entropy_ref(logits.view(-1, logits.shape[-1]), labels.reshape(-1), ignore_index)


# ----------------------------------------------------------------------------
# Linear / Embedding with direct weight-gradient delivery
# ----------------------------------------------------------------------------
# Transposed weight copies.  hipBLASLt runs Y = X W^T (the forward, "NT") at
# ~1.5 PF/s on MI355X but dX = dY W ("NN") 10-30 % slower on every Llama
# shape (profiles/r01_gemm_layouts.jsonl); with a [in, out] copy W^T the input
# gradient becomes dY (W^T)^T, the fast NT form again.  The copy is refreshed
# by an LDS-tiled HIP transpose (edl_transpose_bf16) in the first forward after
# the parameters may have changed — FlatParams.zero_grad() starts a new
# generation, and every parameter mutation (optimizer, state sync, restore)
# happens between steps — so it costs one 4 B/element pass per step (~6 ms for
# Llama-3-8B) and 2 B/param of HBM.  EDL_WT_CACHE=0 disables it.
_WT_GEN = [0]
_WT_ON = os.environ.get("EDL_WT_CACHE", "1") != "0"
# [bytes the transposed copies may still take, weight generation it was measured in]: measured
# from free HBM at first use and again (once per generation) when a copy does not fit -- copies of
# dead weights give their memory back, and a hot standby that measured it beside a live worker
# (utils/vram.py) sees more once it has taken over
_WT_BUDGET: list = [None, -1]
# Batched refresh: at the first use of a new generation every stale cached copy on that device is
# re-transposed in ONE launch (edl_transpose_bf16_multi) instead of one small launch per weight at
# its first use (a BERT-large weight is 64-256 tiles: 9.4 us per 1024 x 1024 transpose alone).
# EDL_WT_BATCH=0: per-weight refresh.
_WT_BATCH = os.environ.get("EDL_WT_BATCH", "1") != "0"
_WT_ALL: list = []            # weakrefs of every weight holding a cached copy
_WT_DESC: dict = {}           # device -> (key, device descriptor tensor, tiles)


def _refresh_stale_wt(w: torch.Tensor) -> bool:
    """Re-transpose every stale cached copy on w's device in one launch; False when only w is
    stale (the caller's single transpose is as good)."""
    gen, live, stale = _WT_GEN[0], [], []
    for ref in _WT_ALL:
        t = ref()
        if t is None:
            continue
        live.append(ref)
        if t.device == w.device and t._edl_wt_gen != gen:
            stale.append(t)
    _WT_ALL[:] = live
    if len(stale) <= 1:
        return False
    key = tuple((t.data_ptr(), t._edl_wt.data_ptr(), t.shape[0], t.shape[1]) for t in stale)
    ent = _WT_DESC.get(w.device)
    if ent is None or ent[0] != key:
        rows, tiles = [], 0
        for t in stale:
            R, C = t.shape
            tx = (C + 127) // 128
            rows.append([t.data_ptr(), t._edl_wt.data_ptr(), (R << 32) | C, (tiles << 32) | tx])
            tiles += tx * ((R + 127) // 128)
        ent = (key, torch.tensor(rows, dtype=torch.int64).to(w.device), tiles)
        _WT_DESC[w.device] = ent
    _native.kernels().check("edl_transpose_bf16_multi", ent[1].data_ptr(), len(stale), ent[2],
                            _native.stream_of(w))
    for t in stale:
        t._edl_wt_gen = gen
    return True


def new_weight_generation() -> None:
    _WT_GEN[0] += 1


def _wt_of(w: torch.Tensor):
    if not (_WT_ON and w.is_cuda and w.dtype == torch.bfloat16 and w.dim() == 2 and w.is_contiguous()
            and w.shape[0] % 8 == 0 and w.shape[1] % 8 == 0):
        return None
    wt = getattr(w, "_edl_wt", None)
    if wt is None:
        gen = _WT_GEN[0]
        if getattr(w, "_edl_wt_skip", None) == gen:
            return None
        # HBM budget: the copies never take the last EDL_WT_RESERVE_GB (default 48) of free memory
        # (activations of the first step still have to fit); weights beyond it keep the NN dgrad
        need = w.numel() * w.element_size()
        if _WT_BUDGET[0] is None or (need > _WT_BUDGET[0] and _WT_BUDGET[1] != gen):
            free, _ = torch.cuda.mem_get_info(w.device)
            _WT_BUDGET[0] = free - float(os.environ.get("EDL_WT_RESERVE_GB", 48)) * 2**30
            _WT_BUDGET[1] = gen
        if need > _WT_BUDGET[0]:
            w._edl_wt_skip = gen      # retried in a later generation, against a fresh measurement
            return None
        _WT_BUDGET[0] -= need
        wt = torch.empty(w.shape[1], w.shape[0], dtype=w.dtype, device=w.device)
        w._edl_wt = wt
        w._edl_wt_gen = -1
        _WT_ALL.append(weakref.ref(w))
    if w._edl_wt_gen != _WT_GEN[0] and not (_WT_BATCH and _refresh_stale_wt(w)):
        _native.kernels().check("edl_transpose_bf16", w.data_ptr(), wt.data_ptr(), w.shape[0], w.shape[1],
                                _native.stream_of(w))
        w._edl_wt_gen = _WT_GEN[0]
    return wt


# Weight gradients in NT form.  dW = dY^T X is a "TN" GEMM, 15-35 % slower in
# hipBLASLt than the NT form dW = (dY^T) (X^T)^T on contiguous transposed
# activations (profiles/r01_gemm_nt_wgrad.jsonl).  The two LDS-tiled transposes
# cost less than that gap when the input width K is small next to the output
# width (qkv, o, gate_up, lm_head: net -0.14 / -0.02 / -0.34 / -1.9 ms per
# 16k-token micro-batch); for wide inputs (down-proj, K = 14336) the X
# transpose eats the gain, so those keep the TN call.  EDL_NT_WGRAD=0 disables.
_NT_WGRAD = os.environ.get("EDL_NT_WGRAD", "1") != "0"
_NT_WGRAD_MAX_K = 8192
# fused MLP (SwiGLU kernels emit the transposed wgrad operands); EDL_MLP_FUSED=0 -> generic path
_MLP_FUSED = os.environ.get("EDL_MLP_FUSED", "1") != "0"
# the gate/up input gradient dX = dGU W_gu (K = 2 x ffn) on the hand-written 8-phase NT GEMM
# (csrc/kernels/gemm_nt.hip, group 4): 1,569-1,585 vs hipBLASLt's 1,517-1,527 TF/s at Llama-3-8B
# (profiles/r06_gemm_nt8.md); every other shape stays with hipBLASLt.  EDL_GEMM_NT8_DGRAD=0 disables.
_NT8_DGRAD = os.environ.get("EDL_GEMM_NT8_DGRAD", "1") != "0"


def _dgrad_gu(dgu: torch.Tensor, wt_gu, w_gu) -> torch.Tensor:
    if wt_gu is None:
        return torch.mm(dgu, w_gu)
    if _NT8_DGRAD and dgu.shape[1] % 128 == 0:
        from easydl_amd.ops import gemm
        if gemm.supported(dgu, wt_gu):
            return gemm.gemm_nt(dgu, wt_gu, group_m=4, kernel="nt8")
    return torch.mm(dgu, wt_gu.t())


def _transposed(t: torch.Tensor) -> torch.Tensor:
    t = t.contiguous()
    out = torch.empty(t.shape[1], t.shape[0], dtype=t.dtype, device=t.device)
    _native.kernels().check("edl_transpose_bf16", t.data_ptr(), out.data_ptr(), t.shape[0], t.shape[1],
                            _native.stream_of(t))
    return out


def _transposed_colsum(t: torch.Tensor) -> tuple[torch.Tensor, torch.Tensor, int]:
    """(t^T, [G, cols] fp32 column-sum partials, G) in one pass over t: the bias gradient
    rides on the transpose the NT weight-gradient GEMM needs anyway."""
    t = t.contiguous()
    k = _native.kernels()
    out = torch.empty(t.shape[1], t.shape[0], dtype=t.dtype, device=t.device)
    G = k("edl_transpose_tiles", t.shape[0])
    partial = torch.empty(G, t.shape[1], dtype=torch.float32, device=t.device)
    k.check("edl_transpose_colsum_bf16", t.data_ptr(), out.data_ptr(), partial.data_ptr(), t.shape[0], t.shape[1],
            _native.stream_of(t))
    return out, partial, G


def _nt_wgrad_ok(dy2: torch.Tensor, x2: torch.Tensor) -> bool:
    return (_NT_WGRAD and dy2.is_cuda and dy2.dtype == torch.bfloat16 and x2.dtype == torch.bfloat16
            and x2.shape[1] <= _NT_WGRAD_MAX_K and dy2.shape[0] % 8 == 0 and dy2.shape[1] % 8 == 0
            and x2.shape[1] % 8 == 0)


# Weight gradients from the row-major operands (csrc/kernels/gemm_tn.hip): dW = dY^T X
# read straight from dY [M, N] and X [M, J] through transposing LDS reads, so the
# backward writes no transposed copies at all (no dY / X transposes, the MLP kernels
# drop their h^T / d(gate_up)^T / du^T outputs).  Applies when N % 128 == 0 and
# J % 256 == 0.  Measured per shape at M = 16384 (profiles/r03_gemm_tn_ab.md): it beats
# hipBLASLt NT + the two transposes on every BERT-large weight (N*J <= 4.2 M: 0.05-0.14 ms
# vs 0.08-0.20 ms) and loses on the Llama-3-8B ones (N*J >= 16.8 M: its 256 x 256 kernel
# runs 1.1-1.2 PF/s against hipBLASLt NT's 1.4-1.6, and the step is slower with any of them
# on it), so by default ("auto") it takes weights of at most EDL_WGRAD_TN_MAX_ELEMS (8 M)
# elements.  EDL_WGRAD_TN=1: every
# eligible weight; 0: never (NT form on transposed copies).
_WGRAD_TN = os.environ.get("EDL_WGRAD_TN", "auto")
_WGRAD_TN_MAX = int(os.environ.get("EDL_WGRAD_TN_MAX_ELEMS", 8 << 20))
# EDL_WGRAD_TN_WIDE_J > 0: also weights whose input is at least that wide (the NT form would
# transpose a wide X).  Off by default: for Llama-3-8B's down projection (J = 14336) the TN
# kernel wins in isolation (1.73 ms vs NT 1.67 + 0.23 ms of transposes) but the step ran
# 2,874 vs 2,791 ms with it (profiles/r03_gemm_tn_ab.md).
_WGRAD_TN_WIDE = int(os.environ.get("EDL_WGRAD_TN_WIDE_J", 0))


def _tn_dims(t: torch.Tensor, N: int, J: int) -> bool:
    """The TN kernel takes dW [N, J] for activations like ``t`` (bf16 on the GPU)."""
    wide = 0 < _WGRAD_TN_WIDE <= J
    if _WGRAD_TN == "0" or (_WGRAD_TN == "auto" and N * J > _WGRAD_TN_MAX and not wide):
        return False
    return t.is_cuda and t.dtype == torch.bfloat16 and N % 128 == 0 and J % 256 == 0


def _tn_ok(dy2: torch.Tensor, x2: torch.Tensor) -> bool:
    return (_tn_dims(dy2, dy2.shape[1], x2.shape[1]) and x2.dtype == torch.bfloat16
            and dy2.dim() == 2 and x2.dim() == 2 and dy2.shape[0] == x2.shape[0]
            and dy2.is_contiguous() and x2.is_contiguous()
            and dy2.data_ptr() % 16 == 0 and x2.data_ptr() % 16 == 0)


def gemm_tn(dy2: torch.Tensor, x2: torch.Tensor, out: torch.Tensor | None = None, accumulate: bool = False):
    """``dy2^T @ x2`` ([M, N]^T [M, J] -> [N, J]) by the HIP TN kernel, written into (or
    accumulated onto) ``out`` (bf16 or fp32, contiguous) or a new bf16 tensor."""
    k = _native.kernels()
    M, N = dy2.shape
    J = x2.shape[1]
    if out is None:
        out = torch.empty(N, J, dtype=dy2.dtype, device=dy2.device)
        accumulate = False
    if out.dtype not in (torch.bfloat16, torch.float32) or not out.is_contiguous() or out.numel() != N * J:
        raise ValueError("gemm_tn: out must be a contiguous bf16/fp32 [N, J] tensor")
    nws = k.raw("edl_gemm_tn_ws_bytes")(M, N, J)
    ws = torch.empty(nws // 4, dtype=torch.float32, device=dy2.device) if nws else None
    k.check("edl_gemm_tn", dy2.data_ptr(), x2.data_ptr(), out.data_ptr(), M, N, J,
            int(out.dtype == torch.float32), int(accumulate), _native.ptr(ws), _native.stream_of(dy2))
    return out


def _colsum_partial(t: torch.Tensor) -> tuple[torch.Tensor, int]:
    """[G, cols] fp32 column-sum partials of a bf16 [M, cols] matrix (reduced by edl_colsum)."""
    k = _native.kernels()
    M, C = t.shape
    G = k("edl_colsum_bf16_groups", M)
    part = torch.empty(G, C, dtype=torch.float32, device=t.device)
    k.check("edl_colsum_bf16_partial", t.data_ptr(), M, C, part.data_ptr(), G, _native.stream_of(t))
    return part, G


# Tensor-parallel overlap hooks (parallel/tp.py).  ``out_reduce``: the output of a
# row-parallel GEMM is a partial sum; it is computed in row chunks and each chunk's
# all-reduce starts (on the communicator's stream) while the next chunk's GEMM runs.
# ``dx_reduce``: the input gradient of a column-parallel GEMM is a partial sum; its
# all-reduce starts as soon as dX exists and runs under the weight-gradient GEMM(s).
# Both are ``start(tensor) -> finish()`` callables: ``finish`` orders the compute
# stream after the collective and returns the reduced tensor.
_TP_CHUNK_ROWS = int(os.environ.get("EDL_TP_CHUNK_ROWS", 2048))


def _chunked_reduced_mm(x2, w, start, out=None):
    """``x2 @ w^T`` with each row chunk's all-reduce started behind its GEMM."""
    M = x2.shape[0]
    y = out if out is not None else torch.empty(M, w.shape[0], dtype=x2.dtype, device=x2.device)
    n = max(1, min(8, M // max(8, _TP_CHUNK_ROWS)))
    step = -(-M // n)
    step = -(-step // 8) * 8
    fins = []
    for lo in range(0, M, step):
        hi = min(M, lo + step)
        torch.mm(x2[lo:hi], w.t(), out=y[lo:hi])
        fins.append(start(y[lo:hi]))
    for f in fins:
        f()
    return y


class _LinearFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, b, dx_reduce=None, out_reduce=None, wgrad_side=False, res_grad=None):
        x2 = x.reshape(-1, x.shape[-1])
        ctx.res_grad = None
        if res_grad is not None and dx_reduce is None and ctx.needs_input_grad[0]:
            res_grad.arm()
            ctx.res_grad = res_grad
        if out_reduce is not None:
            if b is not None:
                raise ValueError("row-parallel linear with an output all-reduce takes no bias")
            y = _chunked_reduced_mm(x2, w, out_reduce)
        else:
            y = F.linear(x2, w, b)
        wt = _wt_of(w) if ctx.needs_input_grad[0] else None
        ctx.save_for_backward(x2, w, wt)
        ctx.has_b = b is not None
        ctx.b = b
        ctx.dx_reduce = dx_reduce
        ctx.wgrad_side = wgrad_side
        return y.view(*x.shape[:-1], w.shape[0])

    @staticmethod
    def backward(ctx, dy):
        x2, w, wt = ctx.saved_tensors
        dy2 = dy.reshape(-1, dy.shape[-1])
        dx = None
        fin = None
        if ctx.needs_input_grad[0]:
            dx = gradsink.input_grad_mm(dy2, wt.t() if wt is not None else w, ctx.res_grad,
                                        (*dy.shape[:-1], w.shape[1]))
            if ctx.dx_reduce is not None:
                fin = ctx.dx_reduce(dx)      # runs under the weight-gradient GEMM below
        dw = db = None
        bias_partial = None   # (partial slab, G): bias gradient computed by the dY transpose
        want_db = ctx.has_b and ctx.needs_input_grad[2]
        if ctx.needs_input_grad[1]:
            if _tn_ok(dy2, x2):
                if want_db:
                    bias_partial = _colsum_partial(dy2)
                dw = _deliver_wgrad(w, dy2, x2, side=ctx.wgrad_side, tn=True)
            elif _nt_wgrad_ok(dy2, x2):
                if want_db:
                    dyT, part, G = _transposed_colsum(dy2)
                    bias_partial = (part, G)
                else:
                    dyT = _transposed(dy2)
                a, b_ = dyT, _transposed(x2).t()   # dY^T (contiguous) @ (X^T)^T: NT GEMM
                dw = _deliver_wgrad(w, a, b_, side=ctx.wgrad_side)
            else:
                dw = _deliver_wgrad(w, dy2.t(), x2, side=ctx.wgrad_side)
        if want_db:
            b = ctx.b
            if bias_partial is not None:
                from easydl_amd.ops.norms import _deliver_colsum
                part, G = bias_partial
                g = _deliver_colsum(_native.kernels(), b, part, G, dy2.shape[1], _native.stream_of(dy2))
                if g is not None:
                    db = g.to(b.dtype)
            else:
                g = dy2.sum(0)
                if gradsink.is_flat(b):
                    gradsink.write(b, g)
                else:
                    db = g.to(b.dtype)
        if fin is not None:
            dx = fin()
        return dx, dw, db, None, None, None, None


def linear(x, w, b=None, *, dx_reduce=None, out_reduce=None, wgrad_side=False, res_grad=None):
    """``x @ w^T + b``; ``dx_reduce`` / ``out_reduce``: tensor-parallel overlap hooks (above);
    ``wgrad_side``: the weight-gradient GEMM runs on the side stream, so the collective that
    consumes dX next (sequence parallelism's reduce-scatter) overlaps it; ``res_grad``: a
    :class:`gradsink.ResidualGrad` slot whose parked residual gradient dX accumulates onto."""
    if (_native.use_hip(x) or gradsink.is_flat(w) or dx_reduce is not None or out_reduce is not None
            or res_grad is not None):
        return _LinearFn.apply(x, w, b, dx_reduce, out_reduce, wgrad_side, res_grad)
    return F.linear(x, w, b)


# Weight-gradient GEMMs on a side stream.  dW = dY^T X feeds nothing else in the
# backward, so it can run beside the input-gradient chain: hipBLASLt's Stream-K
# kernels hold every CU with one 256-VGPR / 130 KB-LDS workgroup, which leaves room
# on each SIMD for the chain's memory-bound kernels (transposes, SwiGLU, norms,
# RoPE; <= 84 VGPRs, <= 512 B LDS) to co-run.  The side stream waits for the main
# stream before each GEMM; its operands are record_stream'ed so the allocator does
# not hand their memory back to the main stream early; ElasticDDP launches bucket
# all-reduces behind both streams and joins them in finish().  Opt-in
# (EDL_WGRAD_STREAM=1): measured on MI355X it slows the Llama-3-8B step 2.79 ->
# 3.6-4.1 s (two GEMMs co-running thrash each other) and ties on BERT-large
# (profiles/r02_wgrad_stream_ab.txt), so by default every GEMM stays on the compute stream.
_WGRAD_STREAM = os.environ.get("EDL_WGRAD_STREAM", "0") == "1"
_SIDE: dict = {}    # device index -> side stream
_MAIN: dict = {}    # device index -> the compute stream the side stream last forked from
_JOIN_QUEUED: dict = {}   # device index -> end-of-backward join already queued


def _dev_index(dev: torch.device) -> int:
    return dev.index if dev.index is not None else torch.cuda.current_device()


def pending_streams(device) -> list:
    """Streams besides the current one whose queued work writes gradients (for DDP)."""
    if device is None or torch.device(device).type != "cuda":
        return []
    i = _dev_index(torch.device(device))
    return [s for s in (_MAIN.get(i), _SIDE.get(i)) if s is not None]


def join_side_streams(device) -> None:
    """Make the current stream wait for every queued side-stream weight gradient."""
    if device is None or torch.device(device).type != "cuda":
        return
    i = _dev_index(torch.device(device))
    _JOIN_QUEUED[i] = False   # re-arm the end-of-backward join even if a failed pass dropped it
    side = _SIDE.get(i)
    if side is not None:
        torch.cuda.current_stream(device).wait_stream(side)


def _write_tn(w, dy2, x2):
    g = w.grad
    gemm_tn(dy2, x2, out=g.view(dy2.shape[1], x2.shape[1]), accumulate=not gradsink.is_fresh(w))
    gradsink.commit(w)


def _deliver_wgrad(w, a, b_, side: bool = False, tn: bool = False):
    """dW = a @ b_ into the flat gradient buffer (or returned); ``tn``: a = dY, b_ = X (both
    row-major [M, *]) and dW = a^T b_ by the TN kernel.  ``side``: on the side stream
    (also when EDL_WGRAD_STREAM is off) — used where a collective, not another GEMM, runs
    beside it."""
    if tn and not (gradsink.is_flat(w) and w.grad.dtype in (torch.bfloat16, torch.float32)
                   and w.grad.is_contiguous()):
        return gemm_tn(a, b_)
    write = _write_tn if tn else gradsink.write_mm
    if gradsink.is_flat(w):
        if (_WGRAD_STREAM or side) and a.is_cuda:
            i = _dev_index(a.device)
            main = torch.cuda.current_stream(a.device)
            side = _SIDE.get(i)
            if side is None:
                from easydl_amd.utils.resources import new_stream
                side = _SIDE[i] = new_stream(a.device)   # CU-masked under a Brain CU plan
            _MAIN[i] = main
            side.wait_stream(main)
            with torch.cuda.stream(side):
                write(w, a, b_)
            a.record_stream(side)
            b_.record_stream(side)
            if not _JOIN_QUEUED.get(i):
                # the compute stream waits for the side stream once this backward pass ends, so
                # whatever reads the gradients next (optimizer, clip, tests) is ordered after them
                _JOIN_QUEUED[i] = True

                def _join(i=i, main=main, side=side):
                    _JOIN_QUEUED[i] = False
                    main.wait_stream(side)
                torch.autograd.Variable._execution_engine.queue_callback(_join)
            return None
        write(w, a, b_)
        return None
    return torch.mm(a, b_)


class _SwiGLUMLPFn(torch.autograd.Function):
    """``down(swiglu(gate_up(x)))`` with the weight gradients of both GEMMs in
    hipBLASLt's NT form.  The SwiGLU kernels emit the transposed operands the NT
    form needs: the forward writes h^T (saved instead of h), the backward writes
    d(gate_up)^T next to d(gate_up).  That replaces two separate transposes,
    including the 14336-wide one the generic path skips (down-proj wgrad stayed
    in the 15 % slower TN form there)."""

    @staticmethod
    def forward(ctx, x, w_gu, w_down, dx_reduce=None, out_reduce=None, wgrad_side=False):
        k = _native.kernels()
        x2 = x.reshape(-1, x.shape[-1])
        gu = F.linear(x2, w_gu)
        M, F2 = gu.shape
        Fh = F2 // 2
        # TN weight gradients need h itself; the NT form needs only h^T (saved instead of h).
        # The two GEMMs choose their forms separately (tn_down, tn_gu).
        ctx.tn_down = _tn_dims(x2, w_down.shape[0], Fh)
        ctx.tn_gu = _tn_dims(x2, F2, x2.shape[1])
        h = torch.empty(M, Fh, dtype=gu.dtype, device=gu.device)
        st = _native.stream_of(gu)
        if ctx.tn_down:
            hT = None
            k.check("edl_swiglu_fwd", gu.data_ptr(), h.data_ptr(), M, Fh, st)
        else:
            hT = torch.empty(Fh, M, dtype=gu.dtype, device=gu.device)
            k.check("edl_swiglu_fwd_t", gu.data_ptr(), h.data_ptr(), hT.data_ptr(), M, Fh, st)
        y = _chunked_reduced_mm(h, w_down, out_reduce) if out_reduce is not None else F.linear(h, w_down)
        if not ctx.tn_down:
            del h
            h = hT
        wt_gu = _wt_of(w_gu) if ctx.needs_input_grad[0] else None
        ctx.save_for_backward(x2, gu, h, w_gu, w_down, wt_gu, _wt_of(w_down))
        ctx.dx_reduce = dx_reduce
        ctx.wgrad_side = wgrad_side
        return y.view(*x.shape[:-1], w_down.shape[0])

    @staticmethod
    def backward(ctx, dy):
        k = _native.kernels()
        x2, gu, hs, w_gu, w_down, wt_gu, wt_down = ctx.saved_tensors   # hs: h (TN) or h^T (NT)
        dy2 = dy.reshape(-1, dy.shape[-1]).contiguous()
        M, F2 = gu.shape
        Fh = F2 // 2
        st = _native.stream_of(gu)
        tn = ctx.tn_gu

        def down_wgrad():
            if ctx.tn_down:
                return _deliver_wgrad(w_down, dy2, hs, tn=True)
            return _deliver_wgrad(w_down, _transposed(dy2), hs.t())

        dh = torch.mm(dy2, wt_down.t()) if wt_down is not None else torch.mm(dy2, w_down)
        overlap = ctx.dx_reduce is not None and ctx.needs_input_grad[0]
        dw_down = None
        if not overlap:
            dw_down = down_wgrad()
            del hs
        dgu = torch.empty_like(gu)
        if tn:
            dguT = None
            k.check("edl_swiglu_bwd", dh.data_ptr(), gu.data_ptr(), dgu.data_ptr(), M, Fh, st)
        else:
            dguT = torch.empty(F2, M, dtype=gu.dtype, device=gu.device)
            k.check("edl_swiglu_bwd_t", dh.data_ptr(), gu.data_ptr(), dgu.data_ptr(), dguT.data_ptr(), M, Fh, st)
        del dh
        dx = fin = None
        if ctx.needs_input_grad[0]:
            dx = _dgrad_gu(dgu, wt_gu, w_gu).view(*dy.shape[:-1], w_gu.shape[1])
        if not tn:
            del dgu
        if overlap:
            # tensor parallel: dX's all-reduce runs under BOTH weight-gradient GEMMs
            fin = ctx.dx_reduce(dx)
            dw_down = down_wgrad()
            del hs
        if tn:
            dw_gu = _deliver_wgrad(w_gu, dgu, x2, side=ctx.wgrad_side, tn=True)
        else:
            dw_gu = _deliver_wgrad(w_gu, dguT, _transposed(x2).t(), side=ctx.wgrad_side)
        if fin is not None:
            dx = fin()
        return dx, dw_gu, dw_down, None, None, None


def swiglu_mlp(x, w_gu, w_down, *, dx_reduce=None, out_reduce=None, wgrad_side=False):
    """Llama MLP ``down(silu(gate) * up)`` with ``w_gu`` = [gate; up] stacked on dim 0.
    ``dx_reduce`` / ``out_reduce`` / ``wgrad_side``: tensor-parallel overlap hooks (see
    ``linear``; ``wgrad_side`` applies to the gate/up weight gradient)."""
    x2 = x.reshape(-1, x.shape[-1])
    if (_MLP_FUSED and _native.use_hip(x) and x.dtype == torch.bfloat16 and _nt_wgrad_ok(x2, x2)
            and x2.shape[0] % 8 == 0 and w_gu.shape[0] % 16 == 0):
        return _SwiGLUMLPFn.apply(x, w_gu, w_down, dx_reduce, out_reduce, wgrad_side)
    return linear(swiglu(linear(x, w_gu, dx_reduce=dx_reduce, wgrad_side=wgrad_side)), w_down,
                  out_reduce=out_reduce)


def _bias_grad(k, b, partial, G, cols, stream):
    """Bias gradient from [G, cols] column-sum partials (into the flat buffer, or returned)."""
    from easydl_amd.ops.norms import _deliver_colsum
    g = _deliver_colsum(k, b, partial, G, cols, stream)
    return None if g is None else g.to(b.dtype)


class _GeluMLPFn(torch.autograd.Function):
    """``fc2(gelu_tanh(fc1(x)))`` -- the BERT MLP, biases on both layers -- with both
    weight gradients in hipBLASLt's NT form.  The GELU kernels write the transposed
    operands: the forward writes h^T beside h and saves only h^T (plus fc1's output);
    the backward writes du^T beside du, with the per-tile column sums that make fc1's
    bias gradient in the same pass.  That replaces PyTorch's GELU forward/backward
    kernels, the transpose of h and the transpose + column sum of du."""

    @staticmethod
    def forward(ctx, x, w1, b1, w2, b2, res_grad=None):
        k = _native.kernels()
        x2 = x.reshape(-1, x.shape[-1])
        ctx.res_grad = None
        if res_grad is not None and ctx.needs_input_grad[0]:
            res_grad.arm()
            ctx.res_grad = res_grad
        u = F.linear(x2, w1, b1)
        M, Fd = u.shape
        ctx.tn = _tn_dims(x2, w2.shape[0], Fd) and _tn_dims(x2, Fd, x2.shape[1])
        h = torch.empty_like(u)
        hT = None if ctx.tn else torch.empty(Fd, M, dtype=u.dtype, device=u.device)
        st = _native.stream_of(u)
        k.check("edl_gelu_fwd_t", u.data_ptr(), h.data_ptr(), _native.ptr(hT), M, Fd, st)
        y = F.linear(h, w2, b2)
        hs = h if ctx.tn else hT   # TN weight gradients read h itself, the NT form h^T
        del h
        wt1 = _wt_of(w1) if ctx.needs_input_grad[0] else None
        ctx.save_for_backward(x2, u, hs, w1, w2, wt1, _wt_of(w2))
        ctx.b1, ctx.b2 = b1, b2
        return y.view(*x.shape[:-1], w2.shape[0])

    @staticmethod
    def backward(ctx, dy):
        k = _native.kernels()
        x2, u, hs, w1, w2, wt1, wt2 = ctx.saved_tensors   # hs: h (TN) or h^T (NT)
        dy2 = dy.reshape(-1, dy.shape[-1]).contiguous()
        M, Fd = u.shape
        st = _native.stream_of(u)
        tn = ctx.tn
        dh = torch.mm(dy2, wt2.t()) if wt2 is not None else torch.mm(dy2, w2)
        if tn:
            part2, G2 = _colsum_partial(dy2)
            dw2 = _deliver_wgrad(w2, dy2, hs, tn=True)
        else:
            dyT, part2, G2 = _transposed_colsum(dy2)
            dw2 = _deliver_wgrad(w2, dyT, hs.t())
            del dyT
        del hs
        db2 = _bias_grad(k, ctx.b2, part2, G2, dy2.shape[1], st) if ctx.needs_input_grad[4] else None
        du = torch.empty_like(u)
        duT = None if tn else torch.empty(Fd, M, dtype=u.dtype, device=u.device)
        G = k("edl_transpose_tiles", M)
        part1 = torch.empty(G, Fd, dtype=torch.float32, device=u.device)
        k.check("edl_gelu_bwd_t", dh.data_ptr(), u.data_ptr(), du.data_ptr(), _native.ptr(duT), part1.data_ptr(),
                M, Fd, st)
        del dh
        dx = None
        if ctx.needs_input_grad[0]:
            dx = gradsink.input_grad_mm(du, wt1.t() if wt1 is not None else w1, ctx.res_grad,
                                        (*dy.shape[:-1], w1.shape[1]))
        if tn:
            dw1 = _deliver_wgrad(w1, du, x2, tn=True)
        else:
            dw1 = _deliver_wgrad(w1, duT, _transposed(x2).t())
        del du
        db1 = _bias_grad(k, ctx.b1, part1, G, Fd, st) if ctx.needs_input_grad[2] else None
        return dx, dw1, db1, dw2, db2, None


def gelu_mlp(x, w1, b1, w2, b2, res_grad=None):
    """BERT MLP ``fc2(gelu_tanh(fc1(x)))`` (biases ``b1``, ``b2``); ``res_grad``: see ``linear``."""
    x2 = x.reshape(-1, x.shape[-1])
    if (_MLP_FUSED and _native.use_hip(x) and x.dtype == torch.bfloat16 and _nt_wgrad_ok(x2, x2)
            and x2.shape[0] % 8 == 0 and w1.shape[0] % 8 == 0 and b1 is not None and b2 is not None):
        return _GeluMLPFn.apply(x, w1, b1, w2, b2, res_grad)
    return linear(F.gelu(linear(x, w1, b1, res_grad=res_grad), approximate="tanh"), w2, b2)


class _EmbeddingFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, ids, w):
        ctx.save_for_backward(ids)
        ctx.wshape = w.shape
        ctx.w = w
        return F.embedding(ids, w)

    @staticmethod
    def backward(ctx, dy):
        (ids,) = ctx.saved_tensors
        w = ctx.w
        V, d = ctx.wshape
        g = torch.ops.aten.embedding_dense_backward(dy.reshape(-1, d), ids.reshape(-1), V, -1, False)
        if gradsink.is_flat(w):
            gradsink.write(w, g)
            return None, None
        return None, g


def embedding(ids, w):
    if gradsink.is_flat(w):
        return _EmbeddingFn.apply(ids, w)
    return F.embedding(ids, w)
