"""Live kernel-mix signal (utils/kmix.py) and what the Brain does with it."""
import time

import pytest

import torch

from easydl_amd.api.spec import Resource, ResourcePlan, RoleResource
from easydl_amd.brain.collectors import GpuInfo, NodeInventory
from easydl_amd.brain.planner import JobFeatures, Planner
from easydl_amd.utils.kmix import KernelMixMeter
from easydl_amd.utils.metrics import cu_count


def _inv():
    return NodeInventory(gpus=[GpuInfo(i, "gfx950", 256, 288.0, busy_pct=90) for i in range(8)], cpus=128,
                         host_mem_gb=2048)


def _plan():
    return ResourcePlan(roles={"worker": RoleResource(4, Resource(gpu=1))}, bucket_mb=128.0)


def test_meter_splits_phase_time_by_class_on_the_host():
    m = KernelMixMeter("cpu", window_s=30)
    assert m.snapshot() is None
    with m.phase("compute"):
        time.sleep(0.03)
    with m.phase("memory"):
        time.sleep(0.01)
    s = m.snapshot()
    assert s["source"] == "host-timer" and s["phases"] == 2
    assert 0.6 < s["compute_frac"] < 0.9 and abs(s["compute_frac"] + s["memory_frac"] - 1) < 1e-3


def test_meter_forgets_phases_older_than_its_window():
    m = KernelMixMeter("cpu", window_s=0.05)
    with m.phase("memory"):
        pass
    time.sleep(0.1)
    assert m.snapshot() is None


def test_measured_cu_sensitivity_gives_a_bandwidth_bound_rank_a_cu_plan_once():
    """A rank whose probe measured almost no slowdown on half the CUs (HBM-bound: a PS applying
    AdamW) gets a CU slice; once it runs on that slice (its metrics report the CUs) the Brain
    does not plan it again; a rank that slows down ~2x on half the CUs keeps the whole GPU;
    CPU-hosted roles get no CU plan at all.  No role or phase label enters the decision."""
    ps_mix = {"compute_frac": 0.93, "memory_frac": 0.07, "gpu_s": 3.0, "source": "hip-events",
              "cu_sensitivity": 0.03}
    tr_mix = {"compute_frac": 0.93, "memory_frac": 0.07, "gpu_s": 30.0, "source": "hip-events",
              "cu_sensitivity": 0.92}
    metrics = {"job-ps-0:11": {"role": "worker", "device": "cuda", "gpu_mix": ps_mix, "cu": None},
               "job-worker-0:12": {"role": "worker", "device": "cuda", "gpu_mix": tr_mix, "step_time": 1.0},
               "job-ps-1:13": {"role": "ps", "device": "cpu", "gpu_mix": ps_mix, "busy_frac": 0.1, "cpu": 4}}
    nxt = Planner().next_plan(JobFeatures(mode="ps", params=3.3e8), _inv(), _plan(), metrics)
    cu = nxt.per_rank["job-ps-0:11"]["cu"]
    assert 0 < cu < 256 and cu % 8 == 0 and "measured on half the CUs" in nxt.reason
    assert "cu" not in nxt.per_rank.get("job-worker-0:12", {}) and "job-ps-1:13" not in nxt.per_rank
    metrics["job-ps-0:21"] = dict(metrics.pop("job-ps-0:11"), cu=cu)      # the replacement, on its slice
    again = Planner().next_plan(JobFeatures(mode="ps", params=3.3e8), _inv(), _plan(), metrics)
    assert again is None or "job-ps-0:21" not in again.per_rank


def test_ranks_sharing_a_gpu_the_most_sensitive_keeps_every_cu():
    """Two probed ranks on one GPU (the values the GPU test measured on MI355X: a Llama block
    stack 0.45, a GEMV stack 0.23): on a shared GPU only the less sensitive co-tenant is sliced;
    ranks alone on their GPUs each get the slice that keeps them within 5 %."""
    mix = lambda s: {"compute_frac": 0.95, "memory_frac": 0.05, "gpu_s": 2.0, "source": "hip-events",
                     "cu_sensitivity": s}
    metrics = {"w-0:1": {"device": "cuda", "gpu": 0, "gpu_mix": mix(0.45)},
               "w-1:2": {"device": "cuda", "gpu": 0, "gpu_mix": mix(0.23)}}
    nxt = Planner().next_plan(JobFeatures(mode="allreduce", params=1e8, max_workers=2), _inv(), _plan(), metrics)
    assert "cu" not in nxt.per_rank.get("w-0:1", {})
    assert 0 < nxt.per_rank["w-1:2"]["cu"] < 256
    metrics["w-0:1"]["gpu_mix"] = mix(0.40)
    metrics["w-1:2"]["gpu"] = 1                                       # each alone: the 5 % rule for both
    nxt = Planner().next_plan(JobFeatures(mode="allreduce", params=1e8, max_workers=2), _inv(), _plan(), metrics)
    assert nxt.per_rank["w-0:1"]["cu"] < 256 and nxt.per_rank["w-1:2"]["cu"] < nxt.per_rank["w-0:1"]["cu"]


def test_a_phase_label_alone_never_plans_cus():
    """the phase split says where kernels were launched from, not what they do."""
    mix = {"compute_frac": 0.02, "memory_frac": 0.98, "gpu_s": 3.0, "source": "hip-events"}
    metrics = {"job-ps-0:11": {"role": "ps", "device": "cuda", "gpu_mix": mix}}
    nxt = Planner().next_plan(JobFeatures(mode="ps", params=3.3e8), _inv(), _plan(), metrics)
    assert nxt is None or "job-ps-0:11" not in nxt.per_rank


def test_cu_for_sensitivity_keeps_the_slowdown_small():
    p = Planner
    assert p.cu_for_sensitivity(None) is None and p.cu_for_sensitivity(0.9) is None
    assert p.cu_for_sensitivity(0.0) == 64                      # HBM saturates at ~1/4 of the chip
    for s in (0.01, 0.03, 0.1, 0.3):
        c = p.cu_for_sensitivity(s)
        assert c % 8 == 0 and s * (256 / c - 1) <= 0.05 + 1e-9, (s, c)
    assert p.cu_for_sensitivity(0.03) < p.cu_for_sensitivity(0.1) < p.cu_for_sensitivity(0.3)


def test_hbm_plan_from_the_allocator_peak():
    m = {"device": "cuda", "gpu": 0, "hbm_peak_gb": 20.0, "hbm_total_gb": 288.0, "hbm_cap_gb": None}
    nxt = Planner().next_plan(JobFeatures(mode="ps", params=3.3e8), _inv(), _plan(), {"w:1": m})
    assert nxt.per_rank["w:1"]["hbm_gb"] == 25.0 and "HBM cap 25 GB" in nxt.reason
    full = dict(m, hbm_peak_gb=250.0)                           # no headroom: no cap
    again = Planner().next_plan(JobFeatures(mode="ps", params=3.3e8), _inv(), _plan(), {"w:1": full})
    assert again is None or "hbm_gb" not in again.per_rank.get("w:1", {})
    capped = dict(m, hbm_cap_gb=25.0)                           # already running under it
    assert Planner.hbm_for_rank(capped) is None


def test_single_rank_gpu_without_a_probe_uses_amdsmi_activity():
    inv = _inv()
    inv.gpus[3].busy_pct, inv.gpus[3].umc_pct = 95.0, 85.0      # memory controllers busy all along
    inv.gpus[4].busy_pct, inv.gpus[4].umc_pct = 98.0, 20.0      # matrix cores busy, HBM idle-ish
    metrics = {"a:1": {"device": "cuda", "gpu": 3, "gpu_mix": {"compute_frac": 0.9, "source": "hip-events"}},
               "b:2": {"device": "cuda", "gpu": 4, "gpu_mix": {"compute_frac": 0.1, "source": "hip-events"}}}
    nxt = Planner().next_plan(JobFeatures(mode="ps", params=3.3e8), inv, _plan(), metrics)
    assert 0 < nxt.per_rank["a:1"]["cu"] < 256 and "amd-smi" in nxt.reason
    assert "cu" not in nxt.per_rank.get("b:2", {})


def test_busy_cpu_parameter_server_gets_more_cores_up_to_the_cap():
    from easydl_amd.brain.planner import BrainConfig
    metrics = {"job-ps-0:5": {"role": "ps", "device": "cpu", "busy_frac": 0.9, "cpu": 4}}
    p = Planner(BrainConfig(ps_busy_high=0.75, ps_cpu_max=6))
    nxt = p.next_plan(JobFeatures(mode="ps", params=1e5), _inv(), _plan(), metrics)
    assert nxt.per_rank["job-ps-0:5"]["cpu"] == 6
    metrics["job-ps-0:5"]["cpu"] = 6
    assert Planner(BrainConfig(ps_busy_high=0.75, ps_cpu_max=6)).next_plan(
        JobFeatures(mode="ps", params=1e5), _inv(), _plan(), metrics) is None
    metrics["job-ps-0:5"].update(cpu=2, busy_frac=0.3)
    assert p.next_plan(JobFeatures(mode="ps", params=1e5), _inv(), _plan(), metrics) is None


def test_cu_count_of_operator_masks():
    from easydl_amd.operator.reconciler import cu_mask_hex
    assert cu_count(None) is None and cu_count(cu_mask_hex(64)) == 64 and cu_count(cu_mask_hex(256)) == 256


def test_trainer_publishes_its_live_mix_with_its_metrics(tmp_path):
    from easydl_amd.trainer.context import TrainerContext
    from easydl_amd.trainer.data import SyntheticTokens
    from easydl_amd.trainer.elastic import ElasticTrainer
    from easydl_amd.models.llama import Llama, get_config
    cfg = get_config("llama-tiny")
    tr = ElasticTrainer(lambda d: Llama(cfg, device=d, dtype=torch.float32), global_batch=2, micro_batch=1,
                        device="cpu", ctx=TrainerContext(job="km", run_dir=str(tmp_path)))
    tr.metrics.every = 5
    tr.fit(lambda m, b: m(*b), SyntheticTokens(cfg.vocab_size, 32, num_samples=64), num_steps=5)
    mix = tr.metrics.last["gpu_mix"]
    assert mix["phases"] == 10 and mix["compute_frac"] > 0.5 and tr.metrics.last["role"] == "worker"


@pytest.mark.gpu
def test_meter_reads_hip_event_times_without_synchronising(cuda):
    m = KernelMixMeter(cuda, window_s=60)
    a = torch.randn(8192, 8192, device=cuda, dtype=torch.bfloat16)
    x = torch.randn(64 << 20, device=cuda)
    for _ in range(3):
        with m.phase("compute"):
            for _ in range(4):
                a @ a
        with m.phase("memory"):
            for _ in range(4):
                x.mul_(1.0001)
    torch.cuda.synchronize(cuda)
    s = m.snapshot()
    assert s["source"] == "hip-events" and s["phases"] == 6 and s["gpu_s"] > 0
    # 4 x 1.1 TFLOP of MFMA work vs 4 x 512 MB of streaming: mostly compute
    assert 0.5 < s["compute_frac"] < 1.0


@pytest.mark.gpu
def test_cu_probe_separates_matrix_core_work_from_streaming(cuda):
    """The CU-sensitivity probe on real kernels: GEMMs on half the CUs take up to 2x longer (s
    0.55-0.7 measured: half the chip clocks higher), a streaming update changes much less (s
    0.17-0.31: half the CUs nearly saturate HBM) -- measured, not labelled."""
    out = {}
    a = torch.randn(8192, 8192, device=cuda, dtype=torch.bfloat16)
    x = torch.randn(256 << 20, device=cuda)
    work = {"gemm": lambda: [a @ a for _ in range(4)], "stream": lambda: [x.mul_(1.0001) for _ in range(4)]}
    for name, fn in work.items():
        m = KernelMixMeter(cuda, window_s=60, probe_every=0)
        for i in range(12):
            with m.phase("compute", probe=m.probe_due(i) if i in (4, 6, 8, 10) else False):
                fn()
            if i in (3, 5, 7, 9):
                m.request_probe()
        torch.cuda.synchronize(cuda)
        out[name] = m.cu_sensitivity()
    print(f"\n[cu-probe] {out}")
    assert out["gemm"]["probes"] == 4 and out["stream"]["probes"] == 4
    assert out["gemm"]["s"] > 0.45, out
    assert out["stream"]["s"] < 0.4, out
    assert out["gemm"]["s"] > out["stream"]["s"] + 0.15, out
