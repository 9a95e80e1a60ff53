"""easydl_amd/ops/conv.py: 1x1 convolutions as GEMMs over the channels-last pixel
matrix and MIOpen convolutions with their weight gradient delivered straight into the
flat gradient buffer (no autograd accumulate): same values as F.conv2d."""
import pytest
import torch
import torch.nn.functional as F

from easydl_amd.ops.conv import _Conv1x1Fn, _ConvFn, conv2d
from easydl_amd.parallel.flat import FlatParams


def _ref(x, w, stride=1, padding=0):
    xr, wr = x.detach().clone().requires_grad_(), w.detach().clone().requires_grad_()
    y = F.conv2d(xr, wr, None, stride, padding)
    return y, xr, wr


@pytest.mark.parametrize("flat", [False, True])
def test_conv1x1_gemm_matches_conv2d_cpu(flat):
    torch.manual_seed(0)
    conv = torch.nn.Conv2d(24, 40, 1, bias=False)
    x = torch.randn(3, 24, 5, 7).to(memory_format=torch.channels_last).requires_grad_()
    w0 = conv.weight.detach().clone()
    if flat:
        fp = FlatParams(conv)
        fp.zero_grad()
    y = _Conv1x1Fn.apply(x, conv.weight)
    dy = torch.randn_like(y)
    y.backward(dy)
    yr, xr, wr = _ref(x, w0)
    yr.backward(dy)
    torch.testing.assert_close(y, yr, rtol=1e-5, atol=1e-5)
    torch.testing.assert_close(x.grad, xr.grad, rtol=1e-5, atol=1e-5)
    torch.testing.assert_close(conv.weight.grad, wr.grad, rtol=1e-5, atol=1e-5)
    if flat:   # delivered into the flat buffer, not through autograd accumulation
        assert conv.weight.grad.data_ptr() == fp.groups[0].grad.data_ptr() and not fp.saw_autograd


def test_conv_direct_wgrad_accumulates_over_micro_batches_cpu():
    torch.manual_seed(1)
    conv = torch.nn.Conv2d(8, 16, 3, stride=2, padding=1, bias=False)
    w0 = conv.weight.detach().clone()
    fp = FlatParams(conv)
    fp.zero_grad()
    xs = [torch.randn(2, 8, 9, 9) for _ in range(2)]
    ref = torch.zeros_like(w0)
    for x in xs:   # two micro-batches: the first write copies, the second adds
        y = _ConvFn.apply(x, conv.weight, [2, 2], [1, 1])
        y.sum().backward()
        yr, _, wr = _ref(x, w0, 2, 1)
        yr.sum().backward()
        ref += wr.grad
    torch.testing.assert_close(conv.weight.grad, ref, rtol=1e-5, atol=1e-5)
    assert not fp.saw_autograd


@pytest.mark.gpu
def test_resnet_conv_ops_match_reference_gpu(cuda):
    """bf16 channels-last on the GPU: the 1x1 GEMM path and the MIOpen path with direct
    weight-gradient delivery agree with F.conv2d (fp32 reference of the same bf16 data)."""
    torch.manual_seed(0)
    for k, s, p, cin, cout in [(1, 1, 0, 64, 256), (3, 1, 1, 64, 64), (1, 2, 0, 256, 512), (7, 2, 3, 3, 64)]:
        conv = torch.nn.Conv2d(cin, cout, k, s, p, bias=False, device=cuda, dtype=torch.bfloat16)
        conv = conv.to(memory_format=torch.channels_last)
        w0 = conv.weight.detach().float()
        fp = FlatParams(conv)
        fp.zero_grad()
        x = torch.randn(4, cin, 28, 28, device=cuda, dtype=torch.bfloat16).to(memory_format=torch.channels_last)
        xg = x.detach().requires_grad_()
        y = conv2d(xg, conv)
        dy = torch.randn_like(y)
        y.backward(dy)
        xr = x.detach().float().requires_grad_()
        wr = w0.clone().requires_grad_()
        yr = F.conv2d(xr, wr, None, s, p)
        yr.backward(dy.float())
        for got, want in ((y.float(), yr), (xg.grad.float(), xr.grad), (conv.weight.grad.float(), wr.grad)):
            err = ((got - want).abs().max() / want.abs().max()).item()
            assert err < 2e-2, (k, s, err)
        assert not fp.saw_autograd
