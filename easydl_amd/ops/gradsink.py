"""Gradient delivery protocol between fused ops and flat gradient buffers.

Parameters managed by :class:`easydl_amd.parallel.flat.FlatParams` live as views
into one contiguous buffer and their ``.grad`` is preset to a view of one flat
gradient buffer.  A fused op's backward can then write the weight gradient
*directly* into that view (``torch.mm(..., out=grad)`` on the first
micro-batch, ``addmm_`` afterwards) instead of returning it to autograd, which
would allocate a temporary and run an extra accumulate pass over it.

After writing, the op calls :func:`commit`, which fires the parameter's ready
callback — that is how :class:`easydl_amd.parallel.ddp.ElasticDDP` learns a
bucket is complete and launches its all-reduce while backward continues.

Parameters not managed by a flat buffer fall back to ordinary autograd
accumulation (the op returns the gradient).
"""
from __future__ import annotations

import torch


def is_flat(p: torch.Tensor) -> bool:
    return getattr(p, "_edl_flat", False) and p.grad is not None


def await_shadow(p: torch.Tensor) -> None:
    """The caller's stream is about to write ``p``'s gradient: order it after whatever still
    reads p's gradient group on another stream -- the device -> host copy into the host gradient
    shadow (utils/gshadow.py), or the optimizer update overlapping the next step's forward
    (ElasticTrainer._opt_overlap)."""
    ev = getattr(p, "_edl_wait", None)
    if ev is not None:
        p._edl_wait = None
        torch.cuda.current_stream(p.device).wait_event(ev)


def is_fresh(p: torch.Tensor) -> bool:
    """True: the next write overwrites ``p``'s gradient (first of the accumulation window).
    Every direct writer asks this right before it writes, so this is also where the write waits
    for a pending gradient-shadow copy of it (await_shadow)."""
    await_shadow(p)
    return getattr(p, "_edl_fresh", True)


def commit(p: torch.Tensor) -> None:
    p._edl_fresh = False
    cb = getattr(p, "_edl_ready_cb", None)
    if cb is not None:
        cb(p)


def write(p: torch.Tensor, g: torch.Tensor) -> None:
    """Deliver a computed gradient ``g`` (same numel as ``p``) into ``p.grad``."""
    tgt = p.grad
    g = g.reshape(tgt.shape)
    if is_fresh(p):
        tgt.copy_(g)
    else:
        tgt.add_(g.to(tgt.dtype))
    commit(p)


class ResidualGrad:
    """Hand-off of a residual-path gradient to the GEMM that makes the other gradient of
    the same tensor.

    In a post-norm block ``y = norm(f(x) + x)`` the input ``x`` gets two gradients: the
    norm's residual gradient and ``f``'s first GEMM's input gradient ``dY W``; autograd
    sums them with a separate add kernel.  With a slot shared by the two ops, the norm's
    backward (which always runs first: ``f(x)`` feeds it) parks its residual gradient
    here instead of returning it, and the GEMM accumulates into it in place
    (``r.addmm_(dY, W)``: hipBLASLt with beta = 1), so the add costs only the GEMM
    epilogue's read of ``r``.  A slot serves one forward/backward pass.  The GEMM op arms
    the slot in its forward (it will take the gradient in its backward); the norm uses
    the slot only when it is armed, so a consumer that cannot take it (a fallback path)
    never loses the residual gradient."""

    __slots__ = ("g", "armed")

    def __init__(self):
        self.g = None
        self.armed = False

    def arm(self) -> None:
        self.armed = True

    def put(self, g: torch.Tensor) -> None:
        if self.g is not None:
            raise RuntimeError("ResidualGrad: a residual gradient is already parked (slot reused?)")
        self.g = g

    def take(self):
        g, self.g = self.g, None
        return g


def input_grad_mm(dy2: torch.Tensor, w: torch.Tensor, slot: "ResidualGrad | None", shape) -> torch.Tensor:
    """``dy2 @ w`` (+ the residual gradient parked in ``slot``, accumulated in place)."""
    r = slot.take() if slot is not None else None
    if r is None:
        return torch.mm(dy2, w).view(*shape)
    r2 = r.view(dy2.shape[0], w.shape[1])
    if r2.dtype != dy2.dtype or not r2.is_contiguous():
        return (torch.mm(dy2, w) + r2).view(*shape)
    if r2.is_cuda:
        # the parked tensor is also the gradient another GEMM's weight gradient reads; if that
        # GEMM runs on the side stream (EDL_WGRAD_STREAM / wgrad_side), the in-place update
        # below must not overtake it: order this stream after the side stream's queued work
        from easydl_amd.ops import fused
        side = fused._SIDE.get(fused._dev_index(r2.device))
        if side is not None and side != torch.cuda.current_stream(r2.device):
            torch.cuda.current_stream(r2.device).wait_stream(side)
    r2.addmm_(dy2, w)
    return r2.view(*shape)


def write_mm(p: torch.Tensor, a: torch.Tensor, b: torch.Tensor) -> None:
    """Deliver ``a @ b`` into ``p.grad`` without a temporary when dtypes allow."""
    tgt = p.grad
    tgt2 = tgt.view(a.shape[0], b.shape[1])
    if tgt.dtype == a.dtype:
        if is_fresh(p):
            torch.mm(a, b, out=tgt2)
        else:
            tgt2.addmm_(a, b)
    elif (a.is_cuda and tgt.dtype == torch.float32 and a.dtype == b.dtype == torch.bfloat16
          and tgt2.is_contiguous()):
        # fp32 gradient buffer (grad_dtype=fp32) with bf16 operands: hipBLASLt's bf16 x bf16
        # -> fp32 GEMM writes / accumulates (beta = 1) straight into it, no temporary
        if is_fresh(p):
            torch.ops.aten.mm.dtype_out(a, b, torch.float32, out=tgt2)
        else:
            torch.ops.aten.addmm.dtype_out(tgt2, a, b, torch.float32, out=tgt2)
    else:  # e.g. fp32 gradient buffer with bf16 activations on the CPU
        r = torch.mm(a, b)
        if is_fresh(p):
            tgt2.copy_(r)
        else:
            tgt2.add_(r.to(tgt.dtype))
    commit(p)
