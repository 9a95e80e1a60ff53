"""ResNet-50's 1x1 stride-1 convolutions (NHWC bf16, batch 256): MIOpen (F.conv2d fwd +
bwd, as the model runs today) vs the same math as three hipBLASLt GEMMs (fwd, dgrad,
wgrad in the TN form that writes straight into a gradient buffer).  One JSON line per
shape plus a total; min of 5 timed repetitions after warmup."""
import json
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

SHAPES = [  # (cin, cout, hw, count in the network)
    (64, 64, 56, 1), (64, 256, 56, 4), (256, 64, 56, 2), (256, 128, 56, 1), (128, 512, 28, 4), (512, 128, 28, 3),
    (512, 256, 28, 1), (256, 1024, 14, 6), (1024, 256, 14, 5), (1024, 512, 14, 1), (512, 2048, 7, 4),
    (2048, 512, 7, 2)]


def timeit(fn, reps=5, inner=10):
    fn()
    torch.cuda.synchronize()
    best = 1e9
    for _ in range(reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(inner):
            fn()
        e1.record()
        torch.cuda.synchronize()
        best = min(best, e0.elapsed_time(e1) / inner)
    return best


def main():
    from easydl_amd.ops import conv_tuning
    conv_tuning.install()
    N = 256
    tot_m = tot_g = 0.0
    for cin, cout, hw, cnt in SHAPES:
        x = torch.randn(N, cin, hw, hw, device="cuda", dtype=torch.bfloat16).to(memory_format=torch.channels_last)
        w = (torch.randn(cout, cin, 1, 1, device="cuda", dtype=torch.bfloat16) * 0.05).to(
            memory_format=torch.channels_last)
        dy = torch.randn(N, cout, hw, hw, device="cuda", dtype=torch.bfloat16).to(memory_format=torch.channels_last)
        xr = x.detach().requires_grad_()
        wr = w.detach().requires_grad_()

        def miopen():
            y = F.conv2d(xr, wr)
            xr.grad = wr.grad = None
            y.backward(dy)

        x2 = x.permute(0, 2, 3, 1).reshape(-1, cin)
        dy2 = dy.permute(0, 2, 3, 1).reshape(-1, cout)
        w2 = w.reshape(cout, cin)
        gw = torch.empty(cout, cin, device="cuda", dtype=torch.bfloat16)

        def gemm():
            torch.mm(x2, w2.t())            # fwd  [NHW, cout]
            torch.mm(dy2, w2)               # dgrad [NHW, cin]
            torch.mm(dy2.t(), x2, out=gw)   # wgrad [cout, cin]

        tm, tg = timeit(miopen), timeit(gemm)
        tot_m += cnt * tm
        tot_g += cnt * tg
        print(json.dumps({"cin": cin, "cout": cout, "hw": hw, "count": cnt, "miopen_ms": round(tm, 4),
                          "gemm_ms": round(tg, 4)}), flush=True)
    print(json.dumps({"total_per_step_ms": {"miopen": round(tot_m, 3), "gemm": round(tot_g, 3)}}), flush=True)


if __name__ == "__main__":
    main()
