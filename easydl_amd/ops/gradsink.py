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


def is_fresh(p: torch.Tensor) -> bool:
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


def write_mm(p: torch.Tensor, a: torch.Tensor, b: torch.Tensor) -> None:
    """Deliver ``a @ b`` into ``p.grad`` without a temporary when dtypes allow."""
    tgt = p.grad
    tgt2 = tgt.view(a.shape[0], b.shape[1])
    if tgt.dtype == a.dtype:
        if is_fresh(p):
            torch.mm(a, b, out=tgt2)
        else:
            tgt2.addmm_(a, b)
    else:  # e.g. fp32 gradient buffer with bf16 activations
        r = torch.mm(a, b)
        if is_fresh(p):
            tgt2.copy_(r)
        else:
            tgt2.add_(r.to(tgt.dtype))
    commit(p)
