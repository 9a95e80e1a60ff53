"""Convolutions whose weight gradient goes straight into the flat gradient buffer.

With ``nn.Conv2d`` the weight gradient of every convolution is a fresh tensor
that autograd then ADDS into the parameter's ``.grad`` (a view of the flat
gradient buffer): one extra elementwise launch per convolution per step, and
because a parameter took the autograd path, ``FlatParams.zero_grad`` must
memset the whole gradient buffer every step (profiles/r02_resnet50_kernel_stats.csv:
702 ``CUDAFunctor_add`` launches, 4.3 % of the ResNet-50 step).

* convolutions run on MIOpen (``aten.convolution`` / ``aten.convolution_backward``)
  and the weight gradient is delivered with :func:`gradsink.write` (a copy on the
  first micro-batch instead of an add, and the gradient buffer no longer needs its
  per-step memset);
* ``EDL_CONV1X1_GEMM=1``: 1x1 stride-1 convolutions on channels-last bf16 tensors
  as GEMMs over the [N*H*W, C] pixel matrix (forward, input gradient, weight
  gradient written by :func:`gradsink.write_mm`).  Off by default: hipBLASLt on
  these skinny shapes (K or N = 64..2048 against 0.2-0.8 M pixel rows) took 21.7 ms
  per step against MIOpen's 10.8 ms (profiles/r03_conv1x1_probe.txt), and the
  ResNet-50 step went 34.9 -> 46.8 ms.
"""
from __future__ import annotations

import os

import torch
import torch.nn.functional as F

from easydl_amd.ops import gradsink

_GEMM_1X1 = os.environ.get("EDL_CONV1X1_GEMM", "0") == "1"


class _Conv1x1Fn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w):
        N, C, H, W = x.shape
        cout = w.shape[0]
        x2 = x.permute(0, 2, 3, 1).reshape(-1, C)          # channels-last: a view
        y2 = torch.mm(x2, w.reshape(cout, C).t())
        ctx.save_for_backward(x2, w)
        ctx.nhw = (N, H, W)
        return y2.view(N, H, W, cout).permute(0, 3, 1, 2)   # NCHW shape, channels-last memory

    @staticmethod
    def backward(ctx, dy):
        x2, w = ctx.saved_tensors
        N, H, W = ctx.nhw
        cout, C = w.shape[0], w.shape[1]
        dy2 = dy.contiguous(memory_format=torch.channels_last).permute(0, 2, 3, 1).reshape(-1, cout)
        dx = dw = None
        if ctx.needs_input_grad[0]:
            dx = torch.mm(dy2, w.reshape(cout, C)).view(N, H, W, C).permute(0, 3, 1, 2)
        if ctx.needs_input_grad[1]:
            if gradsink.is_flat(w):
                gradsink.write_mm(w, dy2.t(), x2)
            else:
                dw = torch.mm(dy2.t(), x2).view_as(w)
        return dx, dw


class _ConvFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, stride, padding):
        ctx.save_for_backward(x, w)
        ctx.stride, ctx.padding = stride, padding
        return torch.ops.aten.convolution(x, w, None, stride, padding, [1, 1], False, [0, 0], 1)

    @staticmethod
    def backward(ctx, dy):
        x, w = ctx.saved_tensors
        mask = [ctx.needs_input_grad[0], ctx.needs_input_grad[1], False]
        dx, dw, _ = torch.ops.aten.convolution_backward(dy, x, w, None, ctx.stride, ctx.padding, [1, 1], False,
                                                        [0, 0], 1, mask)
        if dw is not None and gradsink.is_flat(w):
            gradsink.write(w, dw)
            dw = None
        return dx, dw, None, None


def conv2d(x: torch.Tensor, conv: torch.nn.Conv2d) -> torch.Tensor:
    """``conv(x)`` for a bias-free, ungrouped, undilated ``nn.Conv2d`` (ResNet's)."""
    w = conv.weight
    if (not x.is_cuda or conv.bias is not None or conv.groups != 1 or conv.dilation != (1, 1)
            or not isinstance(conv.padding, tuple)):
        return conv(x)
    if (_GEMM_1X1 and conv.kernel_size == (1, 1) and conv.stride == (1, 1) and conv.padding == (0, 0)
            and x.dtype == torch.bfloat16 and w.dtype == torch.bfloat16
            and x.is_contiguous(memory_format=torch.channels_last) and w.is_contiguous()):
        return _Conv1x1Fn.apply(x, w)
    if gradsink.is_flat(w):
        return _ConvFn.apply(x, w, list(conv.stride), list(conv.padding))
    return F.conv2d(x, w, None, conv.stride, conv.padding)
