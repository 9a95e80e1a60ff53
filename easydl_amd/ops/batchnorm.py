"""BatchNorm (+ residual add) (+ ReLU) for channels-last bf16 activations
(HIP kernels in csrc/kernels/batchnorm.hip).

``bn_act(x, bn, residual=None, relu=True)`` computes
``relu(bn(x) + residual)`` with the statistics, running-average update and
affine of the ``nn.BatchNorm2d`` module ``bn`` (fp32 weight, bias and running
buffers; bf16 activations).  On the GPU this is two passes over the activation
forward and two backward; the ResNet bottleneck's separate BatchNorm, casts,
residual add and ReLU kernels disappear.  CPU tensors run the fp32 PyTorch
reference :func:`bn_act_ref` (the CPU test tier and the numerics oracle).
"""
from __future__ import annotations

import os

import torch
import torch.nn.functional as F

from easydl_amd import _native
from easydl_amd.ops import gradsink


def bn_act_ref(x, bn, residual=None, relu=True):
    y = F.batch_norm(x.float(), bn.running_mean, bn.running_var, bn.weight, bn.bias,
                     bn.training, bn.momentum, bn.eps)
    if residual is not None:
        y = y + residual.float()
    if relu:
        y = F.relu(y)
    return y.to(x.dtype)


def _nhwc(t):
    """[N, C, H, W] channels-last (or [M, C]) tensor -> (t, its [M, C] row-major storage view)."""
    if t.dim() == 4:
        if not t.is_contiguous(memory_format=torch.channels_last):
            t = t.contiguous(memory_format=torch.channels_last)
        t2 = t.permute(0, 2, 3, 1).reshape(-1, t.shape[1])
    else:
        t = t2 = t.contiguous()
    if t2.data_ptr() % 16:
        t = t.clone(memory_format=torch.channels_last) if t.dim() == 4 else t.clone()
        return _nhwc(t)
    return t, t2


# A/B switches for the backward's two launch / traffic savings (both on by default):
# EDL_BN_DIRECT_GRADS=0 returns dgamma / dbeta to autograd instead of writing the flat
# buffer; EDL_BN_MASK_FROM_X=0 keeps z and reads it back for the ReLU mask.
_DIRECT_GRADS = os.environ.get("EDL_BN_DIRECT_GRADS", "1") != "0"
_MASK_FROM_X = os.environ.get("EDL_BN_MASK_FROM_X", "1") != "0"
# EDL_BN_RES_HANDOFF=0: autograd sums a block output's two gradients (conv1's input gradient and
# the next block's identity path) with an add kernel instead of the BatchNorm backward reading both
_RES_HANDOFF = os.environ.get("EDL_BN_RES_HANDOFF", "1") != "0"


class _BNActFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, res, w, b, run_mean, run_var, momentum, eps, relu, nbt=None):
        k = _native.kernels()
        x, x2 = _nhwc(x)
        M, C = x2.shape
        G = k("edl_bn_groups", M, C)
        if G <= 0:
            raise ValueError(f"batchnorm kernel: unsupported channel count {C} (needs C % 8 == 0, C <= 2048)")
        if x.dtype != torch.bfloat16 or w.dtype != torch.float32:
            raise TypeError("batchnorm kernel expects bf16 activations and fp32 weight / statistics")
        r2 = None
        # identity-path hand-off: a residual produced by a block-output BatchNorm (one with
        # relu and a residual of its own) takes this op's residual gradient in its backward
        # kernels (dz + dz2) -- no autograd add of the two gradients of the block output
        ctx.res_slot = getattr(res, "_edl_grad_slot", None) if (res is not None and _RES_HANDOFF) else None
        if res is not None:
            res, r2 = _nhwc(res)
        z = torch.empty_like(x)
        dev = x.device
        mean = torch.empty(C, dtype=torch.float32, device=dev)
        rstd = torch.empty(C, dtype=torch.float32, device=dev)
        coef = torch.empty(2 * C, dtype=torch.float32, device=dev)
        part = torch.empty(2 * C * G, dtype=torch.float32, device=dev)
        k.check("edl_bn_fwd_train", x.data_ptr(), _native.ptr(r2), z.data_ptr(), w.data_ptr(), b.data_ptr(),
                run_mean.data_ptr(), run_var.data_ptr(), mean.data_ptr(), rstd.data_ptr(), coef.data_ptr(),
                part.data_ptr(), M, C, momentum, eps, int(relu), _native.ptr(nbt), _native.stream_of(x))
        # ReLU without a residual: the backward recomputes the mask from x and these
        # coefficients (2C floats) instead of keeping and re-reading z
        mx = relu and res is None and _MASK_FROM_X
        ctx.save_for_backward(x, z if relu and not mx else None, w, mean, rstd,
                              coef if mx else None)
        ctx.relu, ctx.has_res = relu, res is not None
        ctx.bn_b = b
        ctx.out_slot = None
        if relu and res is not None and not mx and _RES_HANDOFF:
            ctx.out_slot = z._edl_grad_slot = gradsink.ResidualGrad()
        return z

    @staticmethod
    def backward(ctx, dz):
        k = _native.kernels()
        x, z, w, mean, rstd, fcoef = ctx.saved_tensors
        dz, dz2 = _nhwc(dz)
        x2 = _nhwc(x)[1]
        M, C = x2.shape
        G = k("edl_bn_groups", M, C)
        dev = x.device
        dx = torch.empty_like(x)
        dres = torch.empty_like(x) if ctx.has_res and ctx.needs_input_grad[1] else None
        # weight / bias gradients go straight into flat fp32 gradient views when both are
        # flat-managed (written on the first micro-batch, accumulated after): no per-parameter
        # autograd accumulate launch.  Otherwise they are returned to autograd.
        b = ctx.bn_b
        direct = (_DIRECT_GRADS and gradsink.is_flat(w) and gradsink.is_flat(b) and w.grad.dtype == torch.float32
                  and b.grad.dtype == torch.float32 and gradsink.is_fresh(w) == gradsink.is_fresh(b))
        if direct:
            dw, db, acc = w.grad, b.grad, 0 if gradsink.is_fresh(w) else 1
        else:
            dw = torch.empty(C, dtype=torch.float32, device=dev)
            db = torch.empty(C, dtype=torch.float32, device=dev)
            acc = 0
        coef = torch.empty(3 * C, dtype=torch.float32, device=dev)
        part = torch.empty(2 * C * G, dtype=torch.float32, device=dev)
        extra = ctx.out_slot.take() if ctx.out_slot is not None else None   # the next block's identity grad
        e2 = _nhwc(extra)[1] if extra is not None else None
        k.check("edl_bn_bwd", dz2.data_ptr(), _native.ptr(e2), _native.ptr(z), x.data_ptr(), w.data_ptr(),
                mean.data_ptr(), rstd.data_ptr(), _native.ptr(fcoef), dx.data_ptr(), _native.ptr(dres), dw.data_ptr(),
                db.data_ptr(), coef.data_ptr(), part.data_ptr(), M, C, int(ctx.relu), acc, _native.stream_of(x))
        if dres is not None and ctx.res_slot is not None:
            ctx.res_slot.put(dres)   # summed by the residual's producer (above), not by autograd
            dres = None
        if direct:
            gradsink.commit(w)
            gradsink.commit(b)
            return dx, dres, None, None, None, None, None, None, None, None
        return (dx, dres, dw if ctx.needs_input_grad[2] else None, db if ctx.needs_input_grad[3] else None,
                None, None, None, None, None, None)


def _eval_coef(bn):
    scale = bn.weight.float() * torch.rsqrt(bn.running_var.float() + bn.eps)
    return torch.cat([scale, bn.bias.float() - bn.running_mean.float() * scale]).contiguous()


def bn_act(x, bn: torch.nn.BatchNorm2d, residual=None, relu: bool = True):
    """``relu(bn(x) + residual)`` (residual / relu optional) with ``bn``'s parameters and buffers."""
    if not _native.use_hip(x):
        return bn_act_ref(x, bn, residual, relu)
    if bn.training:
        if bn.momentum is None:
            raise ValueError("bn_act: cumulative moving average (momentum=None) is not supported")
        nbt = bn.num_batches_tracked
        if nbt.device != x.device or nbt.dtype != torch.int64:
            nbt.add_(1)
            nbt = None   # else the statistics kernel counts the batch (no separate launch)
        return _BNActFn.apply(x, residual, bn.weight, bn.bias, bn.running_mean, bn.running_var,
                              float(bn.momentum), float(bn.eps), relu, nbt)
    if torch.is_grad_enabled() and (x.requires_grad or (residual is not None and residual.requires_grad)
                                    or bn.weight.requires_grad):
        # frozen statistics but gradients wanted: differentiable torch ops
        c = _eval_coef(bn)
        C = x.shape[1]
        shape = (1, C, 1, 1) if x.dim() == 4 else (1, C)
        y = x.float() * c[:C].view(shape) + c[C:].view(shape)
        if residual is not None:
            y = y + residual.float()
        return (F.relu(y) if relu else y).to(x.dtype)
    k = _native.kernels()
    x, x2 = _nhwc(x)
    M, C = x2.shape
    r2 = _nhwc(residual)[1] if residual is not None else None
    z = torch.empty_like(x)
    k.check("edl_bn_apply", x.data_ptr(), _native.ptr(r2), z.data_ptr(), _eval_coef(bn).data_ptr(), M, C,
            int(relu), _native.stream_of(x))
    return z
