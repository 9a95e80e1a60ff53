"""RMSNorm / LayerNorm with optional fused residual add (HIP kernels in csrc/kernels/norms.hip).

``add_rmsnorm(x, residual, w)`` returns ``(norm(x + residual) * w, x + residual)``
in ONE pass over the activations — the residual stream of a pre-norm
transformer never takes a separate elementwise add.  The backward fuses the
residual-stream gradient into dx as well.

CUDA tensors run the gfx950 kernels; CPU tensors run the fp32 PyTorch
reference below (used by the CPU test tier and as the numerics oracle).
"""
from __future__ import annotations

import torch

from easydl_amd import _native
from easydl_amd.ops import gradsink


# ----------------------------------------------------------------------------
# references (fp32 math, results cast back to the input dtype)
# ----------------------------------------------------------------------------
def rmsnorm_ref(x, w, eps=1e-5):
    xf = x.float()
    y = xf * torch.rsqrt(xf.pow(2).mean(-1, keepdim=True) + eps) * w.float()
    return y.to(x.dtype)


def layernorm_ref(x, w, b, eps=1e-5):
    return torch.nn.functional.layer_norm(x.float(), (x.shape[-1],), w.float(), b.float(), eps).to(x.dtype)


# ----------------------------------------------------------------------------
# weight-gradient delivery
# ----------------------------------------------------------------------------
def _deliver_colsum(k, p, partial, G, cols, stream):
    """Reduce a [G, cols] fp32 partial slab into p's gradient."""
    if gradsink.is_flat(p):
        g = p.grad
        odt = 0 if g.dtype == torch.bfloat16 else 1
        if g.dtype not in (torch.bfloat16, torch.float32):
            raise TypeError(f"unsupported grad dtype {g.dtype}")
        k.check("edl_colsum", partial.data_ptr(), G, cols, g.data_ptr(), odt, 0 if gradsink.is_fresh(p) else 1,
                stream)
        gradsink.commit(p)
        return None
    out = torch.empty(cols, dtype=torch.float32, device=partial.device)
    k.check("edl_colsum", partial.data_ptr(), G, cols, out.data_ptr(), 1, 0, stream)
    return out.to(p.dtype)


class _NormFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, res, w, b, eps, ln, slot=None):
        k = _native.kernels()
        cols = x.shape[-1]
        if cols % 8 or cols > k("edl_norm_max_cols"):
            raise ValueError(f"norm kernel: unsupported hidden size {cols}")
        if x.dtype != torch.bfloat16 or w.dtype != torch.bfloat16:
            raise TypeError("norm kernel expects bf16 activations and weights")
        x = x.contiguous()
        rows = x.numel() // cols
        y = torch.empty_like(x)
        rstd = torch.empty(rows, dtype=torch.float32, device=x.device)
        mean = torch.empty(rows, dtype=torch.float32, device=x.device) if ln else None
        s = None
        if res is not None:
            res = res.contiguous()
            s = torch.empty_like(x)
        st = _native.stream_of(x)
        # an unused sum output (post-LN BERT drops it) arrives as ds=None instead of a zero-filled tensor
        ctx.set_materialize_grads(False)
        if ln:
            k.check("edl_layernorm_fwd", x.data_ptr(), _native.ptr(res), _native.ptr(s), w.data_ptr(),
                    b.data_ptr(), y.data_ptr(), mean.data_ptr(), rstd.data_ptr(), rows, cols, eps, st)
        else:
            k.check("edl_rmsnorm_fwd", x.data_ptr(), _native.ptr(res), _native.ptr(s), w.data_ptr(), y.data_ptr(),
                    rstd.data_ptr(), rows, cols, eps, st)
        src = s if s is not None else x
        ctx.save_for_backward(src, w, b if ln else None, mean, rstd)
        ctx.ln = ln
        ctx.has_res = res is not None
        ctx.slot = slot if res is not None and slot is not None and slot.armed else None
        if s is not None:
            return y, s
        return y

    @staticmethod
    def backward(ctx, dy, ds=None):
        k = _native.kernels()
        src, w, b, mean, rstd = ctx.saved_tensors
        cols = src.shape[-1]
        rows = src.numel() // cols
        dy = torch.zeros_like(src) if dy is None else dy.contiguous()
        if ds is not None:
            ds = ds.contiguous()
        dx = torch.empty_like(src)
        G = k("edl_norm_bwd_groups", rows, cols)
        pw = torch.empty(G, cols, dtype=torch.float32, device=src.device)
        pb = torch.empty(G, cols, dtype=torch.float32, device=src.device) if ctx.ln else None
        st = _native.stream_of(src)
        if ctx.ln:
            k.check("edl_layernorm_bwd", dy.data_ptr(), src.data_ptr(), w.data_ptr(), mean.data_ptr(),
                    rstd.data_ptr(), _native.ptr(ds), dx.data_ptr(), pw.data_ptr(), pb.data_ptr(), rows, cols, st)
        else:
            k.check("edl_rmsnorm_bwd", dy.data_ptr(), src.data_ptr(), w.data_ptr(), rstd.data_ptr(), _native.ptr(ds),
                    dx.data_ptr(), pw.data_ptr(), rows, cols, st)
        dw = _deliver_colsum(k, w, pw, G, cols, st) if ctx.needs_input_grad[2] else None
        db = None
        if ctx.ln and ctx.needs_input_grad[3]:
            db = _deliver_colsum(k, b, pb, G, cols, st)
        dres = dx if ctx.has_res else None
        if ctx.slot is not None and ctx.needs_input_grad[1]:
            # the residual input's other gradient comes from a GEMM that accumulates onto this one
            ctx.slot.put(dx)
            dres = None
        return dx, dres, dw, db, None, None, None


def rmsnorm(x, w, eps: float = 1e-5):
    if _native.use_hip(x):
        return _NormFn.apply(x, None, w, None, eps, False)
    return rmsnorm_ref(x, w, eps)


def add_rmsnorm(x, residual, w, eps: float = 1e-5):
    """Returns ``(rmsnorm(x + residual) * w, x + residual)``; residual may be None."""
    if residual is None:
        return rmsnorm(x, w, eps), x
    if _native.use_hip(x):
        return _NormFn.apply(x, residual, w, None, eps, False)
    s = x + residual
    return rmsnorm_ref(s, w, eps), s


def layernorm(x, w, b, eps: float = 1e-5):
    if _native.use_hip(x):
        return _NormFn.apply(x, None, w, b, eps, True)
    return layernorm_ref(x, w, b, eps)


def add_layernorm(x, residual, w, b, eps: float = 1e-5, res_grad: gradsink.ResidualGrad | None = None):
    """``(layernorm(x + residual), x + residual)``.  ``res_grad``: a slot shared with the GEMM
    that consumed ``residual`` (see :class:`gradsink.ResidualGrad`) -- the residual's gradient
    is handed to that GEMM's input gradient instead of being summed by autograd."""
    if residual is None:
        return layernorm(x, w, b, eps), x
    if _native.use_hip(x):
        return _NormFn.apply(x, residual, w, b, eps, True, res_grad)
    s = x + residual
    return layernorm_ref(s, w, b, eps), s
