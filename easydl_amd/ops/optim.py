"""Flat-buffer optimizer math: fused AdamW / SGD and the global grad-norm clip.

GPU tensors run the kernels of ``csrc/kernels/optim.hip`` (one launch per flat
group); CPU tensors run the identical math in PyTorch.  The combined gradient
scale ``pre_scale x clip_coef`` stays on the device (``dscale`` = [coef, norm,
nonfinite]) so clipping never synchronises the host.
"""
from __future__ import annotations

import math

import torch

from easydl_amd import _native


def _gdtype(g: torch.Tensor) -> int:
    if g.dtype == torch.bfloat16:
        return 0
    if g.dtype == torch.float32:
        return 1
    raise TypeError(f"unsupported gradient dtype {g.dtype}")


def grad_clip_scale(grads: list[torch.Tensor], max_norm: float, pre_scale: float = 1.0, weights=None,
                    reduce=None) -> torch.Tensor:
    """Return a device tensor [coef, norm, nonfinite] for flat gradient buffers.

    ``norm`` is the L2 norm of ``pre_scale * concat(grads)``; ``coef`` =
    ``pre_scale * min(1, max_norm / norm)`` (``max_norm <= 0`` disables clipping).
    Model-parallel form: ``weights`` scales each buffer's sum of squares (1/tp
    for buffers replicated over the TP group) and ``reduce`` all-reduces the
    total over the group, so every rank clips by the global norm.
    """
    dev = grads[0].device
    if weights is not None or reduce is not None:
        weights = weights or [1.0] * len(grads)
        terms = [grad_clip_scale([g], 0.0, 1.0)[1].double().pow(2) * w for g, w in zip(grads, weights)]
        total = torch.stack(terms).sum().reshape(1)
        if reduce is not None:
            reduce(total)
        norm = (total.sqrt() * pre_scale).float().reshape(())
        bad = (~torch.isfinite(norm)).float()
        coef = torch.tensor(pre_scale, dtype=torch.float32, device=dev)
        if max_norm > 0:
            coef = torch.where(norm > max_norm, pre_scale * (max_norm / (norm + 1e-6)), coef)
        return torch.stack([coef, norm, bad]).float()
    if _native.use_hip(grads[0]):
        k = _native.kernels()
        nparts = [k("edl_sumsq_nparts", g.numel()) for g in grads]
        partial = torch.empty(sum(nparts), dtype=torch.float32, device=dev)
        out = torch.empty(3, dtype=torch.float32, device=dev)
        st = _native.stream_of(grads[0])
        off = 0
        for g, n in zip(grads, nparts):
            k.check("edl_sumsq_partial", g.data_ptr(), _gdtype(g), g.numel(), partial[off:].data_ptr(), st)
            off += n
        k.check("edl_clip_finalize", partial.data_ptr(), off, float(pre_scale), float(max_norm), out.data_ptr(), st)
        return out
    sq = torch.zeros((), dtype=torch.float64, device=dev)
    for g in grads:
        sq += g.double().pow(2).sum()
    norm = (sq.sqrt() * pre_scale).float()
    bad = (~torch.isfinite(norm)).float()
    coef = torch.tensor(pre_scale, dtype=torch.float32, device=dev)
    if max_norm > 0:
        coef = torch.where(norm > max_norm, pre_scale * (max_norm / (norm + 1e-6)), coef)
    return torch.stack([coef, norm, bad])


def adamw_flat_(param16, master, m, v, grad, *, lr, beta1, beta2, eps, weight_decay, step, scale=1.0,
                dscale=None):
    """In-place AdamW over flat buffers.

    ``param16``: bf16 model weights (or None when ``master`` is the parameter),
    ``master``: fp32, ``m``/``v``: fp32, or bf16 (stochastically rounded, deterministic in
    (element, step): see ``edl_adamw_flat_m16``), ``grad``: bf16 or fp32, all the same numel.
    """
    n = master.numel()
    m16 = m.dtype == torch.bfloat16
    if m16 != (v.dtype == torch.bfloat16):
        raise TypeError("m and v must have the same dtype")
    if _native.use_hip(master):
        k = _native.kernels()
        for t in (param16, master, m, v, grad):
            if t is not None and (t.data_ptr() % 16 or not t.is_contiguous()):
                raise ValueError("flat optimizer buffers must be contiguous and 16-byte aligned")
        k.check("edl_adamw_flat_m16" if m16 else "edl_adamw_flat", _native.ptr(param16), master.data_ptr(),
                m.data_ptr(), v.data_ptr(), grad.data_ptr(), _gdtype(grad), n, lr, beta1, beta2, eps, weight_decay,
                int(step), float(scale), _native.ptr(dscale), _native.stream_of(master))
        return
    # reference (same operation order as the kernel / torch.optim.AdamW)
    g = grad.float() * scale
    if dscale is not None:
        if float(dscale[2]) != 0.0:
            return
        g = g * dscale[0]
    bc1 = 1.0 - beta1 ** step
    bc2 = 1.0 - beta2 ** step
    if m16:
        mf = m.float().mul_(beta1).add_(g, alpha=1 - beta1)
        vf = v.float().mul_(beta2).addcmul_(g, g, value=1 - beta2)
        denom = vf.sqrt() / math.sqrt(bc2) + eps
        master.mul_(1 - lr * weight_decay).addcdiv_(mf, denom, value=-lr / bc1)
        base = (int(step) * 0x85EBCA77) & _M32
        m.copy_(bf16_stochastic(mf, (base + 0x27D4EB2F) & _M32))
        v.copy_(bf16_stochastic(vf, (base + 0x165667B1) & _M32))
    else:
        m.mul_(beta1).add_(g, alpha=1 - beta1)
        v.mul_(beta2).addcmul_(g, g, value=1 - beta2)
        denom = v.sqrt() / math.sqrt(bc2) + eps
        master.mul_(1 - lr * weight_decay).addcdiv_(m, denom, value=-lr / bc1)
    if param16 is not None:
        param16.copy_(master)


_M32 = 0xFFFFFFFF


def _mix32(x: torch.Tensor) -> torch.Tensor:
    """lowbias32 on uint32 values held in int64 (products wrap mod 2^64; the low 32 bits are exact)."""
    x = x ^ (x >> 16)
    x = (x * 0x7FEB352D) & _M32
    x = x ^ (x >> 15)
    x = (x * 0x846CA68B) & _M32
    return x ^ (x >> 16)


def bf16_stochastic(x: torch.Tensor, seed: int) -> torch.Tensor:
    """fp32 -> bf16 rounded stochastically with the random bits of element e = mix32(e * golden + seed),
    bit-identical to ``f2bf_sr_bits`` in csrc/kernels/optim.hip (inf / NaN: round to nearest)."""
    flat = x.detach().reshape(-1).float().contiguous()
    e = torch.arange(flat.numel(), dtype=torch.int64, device=flat.device)
    r = _mix32(((e * 0x9E3779B1) & _M32) + seed & _M32) & 0xFFFF
    u = flat.view(torch.int32).to(torch.int64) & _M32
    sr = ((u + r) >> 16) & 0xFFFF
    special = (u & 0x7F800000) == 0x7F800000
    rne = flat.to(torch.bfloat16).view(torch.int16).to(torch.int64) & 0xFFFF
    bits = torch.where(special, rne, sr)
    return bits.to(torch.int32).to(torch.int16).view(torch.bfloat16).reshape(x.shape)


def sgd_flat_(param16, master, mom, grad, *, lr, momentum=0.0, weight_decay=0.0, scale=1.0, dscale=None):
    n = master.numel()
    if _native.use_hip(master):
        k = _native.kernels()
        k.check("edl_sgd_flat", _native.ptr(param16), master.data_ptr(), _native.ptr(mom), grad.data_ptr(),
                _gdtype(grad), n, lr, momentum, weight_decay, float(scale), _native.ptr(dscale),
                _native.stream_of(master))
        return
    g = grad.float() * scale
    if dscale is not None:
        if float(dscale[2]) != 0.0:
            return
        g = g * dscale[0]
    d = g + weight_decay * master
    if mom is not None:
        mom.mul_(momentum).add_(d)
        d = mom
    master.add_(d, alpha=-lr)
    if param16 is not None:
        param16.copy_(master)
