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


def _timed_ms(stream, fn, it=10):
    with torch.cuda.stream(stream):
        for _ in range(2):
            fn()
        torch.cuda.synchronize()
        t = time.perf_counter()
        for _ in range(it):
            fn()
        torch.cuda.synchronize()
    return (time.perf_counter() - t) / it * 1e3


def test_cu_plan_holds_for_every_stream_of_a_rank(cuda, tmp_path, monkeypatch):
    """a CU-planned rank's side streams carry its plan too -- the optimizer update
    overlapping the next forward and the side-stream weight-gradient GEMMs run on the same CUs as
    its compute stream (read back with hipExtStreamGetCUMask), and are slowed like its GEMM."""
    from easydl_amd.models.llama import Llama, get_config
    from easydl_amd.ops import fused
    from easydl_amd.ops.optim import adamw_flat_
    from easydl_amd.trainer.data import SyntheticTokens
    from easydl_amd.trainer.elastic import ElasticTrainer
    cfg = get_config("llama-tiny")
    monkeypatch.setattr(fused, "_WGRAD_STREAM", True)      # weight gradients on the side stream
    monkeypatch.setenv("EDL_OPT_OVERLAP", "1")             # the update's stream (auto: >= 4 groups only)
    monkeypatch.setattr(fused, "_SIDE", {})
    monkeypatch.setattr(fused, "_WT_BATCH", fused._WT_BATCH)
    prev = torch.cuda.current_stream()
    mask = cu_mask_hex(32)
    want = resources.mask_words(mask)[:8]
    try:
        ctx = TrainerContext(job="cu", run_dir=str(tmp_path), cu_mask=mask)
        tr = ElasticTrainer(lambda d: Llama(cfg, device=d), global_batch=4, micro_batch=2, device=cuda, ctx=ctx)
        tr.fit(lambda m, b: m(*b), SyntheticTokens(cfg.vocab_size, 128, num_samples=256), num_steps=3)
        torch.cuda.synchronize()
        streams = {"compute": torch.cuda.current_stream(), "optimizer": tr._opt_stream,
                   "wgrad_side": fused._SIDE.get(cuda.index or 0)}
        for name, s in streams.items():
            assert s is not None, name
            assert resources.stream_cu_mask(s) == want, (name, resources.stream_cu_mask(s), want)
        plain = torch.cuda.Stream()
        assert resources.stream_cu_mask(plain) != want
        # the work on those streams is confined: AdamW (memory-bound) and a weight-gradient-sized GEMM
        n = 1 << 27
        p16 = torch.zeros(n, dtype=torch.bfloat16, device=cuda)
        master, m, v = (torch.zeros(n, dtype=torch.float32, device=cuda) for _ in range(3))
        g = torch.full((n,), 1e-3, dtype=torch.bfloat16, device=cuda)
        upd = lambda: adamw_flat_(p16, master, m, v, g, lr=1e-4, beta1=0.9, beta2=0.95, eps=1e-8,  # noqa: E731
                                  weight_decay=0.1, step=1, dscale=None)
        a = torch.randn(8192, 8192, device=cuda, dtype=torch.bfloat16)
        mm = lambda: a @ a  # noqa: E731
        t = {"adamw_plain": _timed_ms(plain, upd), "adamw_opt_stream": _timed_ms(tr._opt_stream, upd),
             "gemm_plain": _timed_ms(plain, mm), "gemm_side_stream": _timed_ms(streams["wgrad_side"], mm)}
        print(f"\n[cu-plan 32/256 CUs] {t}")
        assert t["adamw_opt_stream"] > 1.5 * t["adamw_plain"], t
        assert t["gemm_side_stream"] > 2.5 * t["gemm_plain"], t
        tr.close()
    finally:
        resources.clear_cu_plan()
        torch.cuda.set_stream(prev)
