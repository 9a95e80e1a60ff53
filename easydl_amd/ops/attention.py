"""Flash attention (csrc/kernels/attention.hip): causal or full, GQA, head_dim 64 or 128, bf16.

Inputs are the ``[B, H, S, D]``-shaped views of token-major ``[B, S, H, D]``
memory that the fused RoPE+QKV kernel produces; the output is returned the
same way, so ``o.transpose(1, 2).reshape(B*S, H*D)`` feeding the output
projection is free.  The forward saves only O and the log-sum-exp (fp32
[B,H,S]); the backward recomputes P tile by tile (dK/dV kernel + dQ kernel,
no float atomics).  ``EDL_ATTN=sdpa`` falls back to PyTorch SDPA (used for
A/B comparisons); other head dims also use SDPA.  Head dim 64 (BERT-large,
Llama-3.2-1B/3B) runs the same kernels instantiated for 128-byte rows.
"""
from __future__ import annotations

import math
import os

import torch
import torch.nn.functional as F

from easydl_amd import _native

# EDL_ATTN_QKV_SPLIT=1: split packed qkv into three tensors before the forward (A/B)
_QKV_SPLIT = os.environ.get("EDL_ATTN_QKV_SPLIT", "0") == "1"


def _bshd(t: torch.Tensor) -> torch.Tensor:
    """[B,H,S,D]-shaped tensor -> contiguous [B,S,H,D] memory (no copy if already laid out so)."""
    return t.transpose(1, 2).contiguous()


class _FlashAttnFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, q, k, v, causal, scale):
        kn = _native.kernels()
        B, H, S, D = q.shape
        KV = k.shape[1]
        qm, km, vm = _bshd(q), _bshd(k), _bshd(v)
        o = torch.empty_like(qm)
        lse = torch.empty(B, H, S, dtype=torch.float32, device=q.device)
        kn.check("edl_attn_fwd", qm.data_ptr(), km.data_ptr(), vm.data_ptr(), o.data_ptr(), lse.data_ptr(), B, S, H,
                 KV, D, 1 if causal else 0, scale, _native.stream_of(q))
        ctx.save_for_backward(qm, km, vm, o, lse)
        ctx.causal, ctx.scale = causal, scale
        return o.transpose(1, 2)

    @staticmethod
    def backward(ctx, do):
        kn = _native.kernels()
        qm, km, vm, o, lse = ctx.saved_tensors
        B, S, H, D = qm.shape
        KV = km.shape[2]
        dom = _bshd(do)
        dq, dk, dv = torch.empty_like(qm), torch.empty_like(km), torch.empty_like(vm)
        delta = torch.empty(2, B, H, S, dtype=torch.float32, device=qm.device)  # (delta, -lse*log2e)
        causal = 1 if ctx.causal else 0
        # fp32 partials when the GQA group is split over workgroups (csrc/kernels/attention.hip dkdv64_plan)
        nws = kn.raw("edl_attn_bwd_ws_bytes")(B, S, H, KV, causal)
        ws = torch.empty(nws // 4, dtype=torch.float32, device=qm.device) if nws else None
        kn.check("edl_attn_bwd", qm.data_ptr(), km.data_ptr(), vm.data_ptr(), o.data_ptr(), dom.data_ptr(),
                 lse.data_ptr(), delta.data_ptr(), dq.data_ptr(), dk.data_ptr(), dv.data_ptr(),
                 ws.data_ptr() if ws is not None else None, B, S, H, KV, D, causal, ctx.scale,
                 _native.stream_of(qm))
        return dq.transpose(1, 2), dk.transpose(1, 2), dv.transpose(1, 2), None, None


class _PackedQKVAttnFn(torch.autograd.Function):
    """Attention over one packed ``[B*S, 3*H*D]`` q|k|v projection (BERT's fused qkv
    Linear).  The forward kernels read q, k and v as row-strided slices of the packed
    tensor (row stride 3*H*D, no split pass); the backward copies q out once (the dK/dV
    kernel stages q and dO tiles with one DMA plan) and reads k / v strided.  The backward
    kernels write dq / dk / dv straight into the slices of one packed gradient, so the qkv
    projection's backward gets its input gradient without the concatenation pass
    autograd's unbind would run.  ``EDL_ATTN_QKV_SPLIT=1`` restores the split of all three."""

    @staticmethod
    def forward(ctx, qkv, B, S, H, causal, scale):
        kn = _native.kernels()
        D = qkv.shape[-1] // (3 * H)
        row = H * D
        st = _native.stream_of(qkv)
        o = torch.empty(B, S, H, D, dtype=qkv.dtype, device=qkv.device)
        lse = torch.empty(B, H, S, dtype=torch.float32, device=qkv.device)
        if _QKV_SPLIT:
            qm, km, vm = (torch.empty(B, S, H, D, dtype=qkv.dtype, device=qkv.device) for _ in range(3))
            kn.check("edl_qkv_split", qkv.data_ptr(), qm.data_ptr(), km.data_ptr(), vm.data_ptr(), B * S, row, st)
            kn.check("edl_attn_fwd", qm.data_ptr(), km.data_ptr(), vm.data_ptr(), o.data_ptr(), lse.data_ptr(), B, S,
                     H, H, D, 1 if causal else 0, scale, st)
            ctx.save_for_backward(qm, km, vm, o, lse)
        else:
            base, es = qkv.data_ptr(), qkv.element_size()
            kn.check("edl_attn_fwd_strided", base, base + row * es, base + 2 * row * es, o.data_ptr(), lse.data_ptr(),
                     B, S, H, H, D, 1 if causal else 0, scale, 3 * row, 3 * row, st)
            ctx.save_for_backward(qkv, o, lse)
        ctx.causal, ctx.scale, ctx.shape = causal, scale, (B, S, H, D)
        return o.view(B * S, H * D)

    @staticmethod
    def backward(ctx, do):
        kn = _native.kernels()
        B, S, H, D = ctx.shape
        row = H * D
        saved = ctx.saved_tensors
        st = _native.stream_of(do)
        if len(saved) == 5:
            qm, km, vm, o, lse = saved
            kptr, vptr, kvs = km.data_ptr(), vm.data_ptr(), row
        else:
            qkv, o, lse = saved
            qm = torch.empty(B, S, H, D, dtype=qkv.dtype, device=qkv.device)
            kn.check("edl_qkv_split", qkv.data_ptr(), qm.data_ptr(), None, None, B * S, row, st)
            es = qkv.element_size()
            kptr, vptr, kvs = qkv.data_ptr() + row * es, qkv.data_ptr() + 2 * row * es, 3 * row
        dom = do.reshape(B, S, H, D).contiguous()
        dqkv = torch.empty(B * S, 3 * row, dtype=qm.dtype, device=qm.device)
        delta = torch.empty(2, B, H, S, dtype=torch.float32, device=qm.device)
        causal = 1 if ctx.causal else 0
        nws = kn.raw("edl_attn_bwd_ws_bytes")(B, S, H, H, causal)
        ws = torch.empty(nws // 4, dtype=torch.float32, device=qm.device) if nws else None
        base, es = dqkv.data_ptr(), dqkv.element_size()
        kn.check("edl_attn_bwd_strided", qm.data_ptr(), kptr, vptr, o.data_ptr(), dom.data_ptr(),
                 lse.data_ptr(), delta.data_ptr(), base, base + row * es, base + 2 * row * es,
                 ws.data_ptr() if ws is not None else None, B, S, H, H, D, causal, ctx.scale, 3 * row, 3 * row, kvs,
                 st)
        return dqkv, None, None, None, None, None


def packed_qkv_attention(qkv: torch.Tensor, B: int, S: int, H: int, causal: bool = False,
                         scale: float | None = None) -> torch.Tensor:
    """``qkv`` [B*S, 3*H*D] (q | k | v per token, multi-head) -> attention output [B*S, H*D]."""
    D = qkv.shape[-1] // (3 * H)
    scale = 1.0 / math.sqrt(D) if scale is None else scale
    if (qkv.is_cuda and D in (64, 128) and qkv.dtype == torch.bfloat16 and qkv.is_contiguous()
            and os.environ.get("EDL_ATTN", "hip") != "sdpa" and os.environ.get("EDL_ATTN_PACKED", "1") != "0"):
        return _PackedQKVAttnFn.apply(qkv, B, S, H, causal, scale)
    q, k, v = (t.transpose(1, 2) for t in qkv.view(B, S, 3, H, D).unbind(2))
    return flash_attention(q, k, v, causal, scale).transpose(1, 2).reshape(B * S, H * D)


def attention_ref(q, k, v, causal=True, scale=None):
    """fp32 reference (GQA by head repetition)."""
    H, KV = q.shape[1], k.shape[1]
    if H != KV:
        k = k.repeat_interleave(H // KV, dim=1)
        v = v.repeat_interleave(H // KV, dim=1)
    return F.scaled_dot_product_attention(q.float(), k.float(), v.float(), is_causal=causal,
                                          scale=scale).to(q.dtype)


def flash_attention(q, k, v, causal: bool = True, scale: float | None = None):
    """q [B,H,S,D], k/v [B,KV,S,D] -> [B,H,S,D]."""
    D = q.shape[-1]
    scale = 1.0 / math.sqrt(D) if scale is None else scale
    if q.is_cuda:
        if D in (64, 128) and q.dtype == torch.bfloat16 and os.environ.get("EDL_ATTN", "hip") != "sdpa":
            return _FlashAttnFn.apply(q, k, v, causal, scale)
        return F.scaled_dot_product_attention(q, k, v, is_causal=causal, scale=scale,
                                              enable_gqa=q.shape[1] != k.shape[1])
    return attention_ref(q, k, v, causal, scale)
