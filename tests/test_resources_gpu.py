"""Brain resource enforcement on the GPU: CU-masked stream + HBM cap; roctx ranges."""
import time

import pytest
import torch

from easydl_amd.operator.reconciler import cu_mask_hex
from easydl_amd.trainer.context import TrainerContext
from easydl_amd.utils import resources, trace

pytestmark = pytest.mark.gpu


def _gemm_ms(n=8192, it=10):
    a = torch.randn(n, n, device="cuda", dtype=torch.bfloat16)
    b = torch.randn(n, n, device="cuda", dtype=torch.bfloat16)
    for _ in range(3):
        a @ b
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(it):
        a @ b
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / it * 1e3


def test_cu_mask_restricts_compute(cuda):
    full = _gemm_ms()
    prev = torch.cuda.current_stream()
    ctx = TrainerContext(cu_mask=cu_mask_hex(32))
    out = resources.apply_plan(ctx, cuda)
    try:
        assert out["cu_stream"] and out["cu_count"] == 32
        masked = _gemm_ms()
        print(f"\n[cu-mask] 256 CUs {full:.2f} ms, 32 CUs {masked:.2f} ms")
        assert masked > 2.5 * full  # 1/8 of the CUs must be clearly slower
    finally:
        torch.cuda.set_stream(prev)


def test_roctx_ranges_do_not_fail(cuda):
    trace.enable(True)
    with trace.range("outer"):
        with trace.range("inner"):
            torch.ones(4, device=cuda).sum().item()
    trace.mark("done")
    trace.enable(False)


def test_amdsmi_telemetry_sees_this_process_hbm_and_power(cuda):
    """Brain telemetry: amd-smi in a child process, matched to the KFD
    inventory by PCI address; the 20 GiB this test holds shows up as HBM in use."""
    import json
    from easydl_amd.brain.collectors import amdsmi_telemetry, kfd_gpus
    assert kfd_gpus(), "KFD topology lists no GPU"
    before = amdsmi_telemetry(kfd_gpus(), window_s=0.0)
    assert before is not None, "amd-smi child failed"
    hold = torch.empty(20 << 30, dtype=torch.uint8, device="cuda")
    torch.cuda.synchronize()
    got = amdsmi_telemetry(kfd_gpus(), window_s=0.3)
    print(json.dumps({"before": [g.__dict__ for g in before], "holding_20GiB": [g.__dict__ for g in got]}))
    assert any((g.mem_used_gb or 0) - (b.mem_used_gb or 0) >= 19 for g, b in zip(got, before))
    assert any(g.power_w for g in got)
    assert all(g.xgmi_read_gbps is None or len(g.xgmi_read_gbps) == 8 for g in got)
    del hold
