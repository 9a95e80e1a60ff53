"""VERDICT r5 Next #7: the Brain decides per-rank CU and HBM plans from measured signals.

Two ranks of one job on ONE GPU: a matrix-core-bound Llama block stack and an HBM-bound batch-1
GEMV stack (tests/helpers/cu_probe_rank.py).  They measure one after the other, as they would on
their own GPUs: a half-CU probe taken while another process saturates the card measures that
process, not the rank (the full GPU tier saw the two signals swap when they ran together).
Both run the same trainer code, so no role and no phase label tells them apart.  Each measures
its CU sensitivity on half its CUs (utils/kmix.py) and its allocator peak; the Planner must give
the HBM-bound rank a CU slice, keep every CU for the more sensitive one (ranks sharing a GPU),
and tighten both HBM caps to their measured peaks."""
import json
import os
import subprocess
import sys

import pytest

from easydl_amd.api.spec import Resource, ResourcePlan, RoleResource
from easydl_amd.brain.collectors import GpuInfo, NodeInventory
from easydl_amd.brain.planner import JobFeatures, Planner

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HELPER = os.path.join(ROOT, "tests", "helpers", "cu_probe_rank.py")


def test_measured_signals_give_different_cu_plans_on_one_gpu(tmp_path):
    env = dict(os.environ, PYTHONPATH=ROOT)
    env.pop("EDL_CU_MASK", None)
    kinds = ("compute", "bandwidth")
    for k in kinds:
        p = subprocess.run([sys.executable, HELPER, k, str(tmp_path / f"{k}.json")], env=env, cwd=ROOT, timeout=240)
        assert p.returncode == 0, k
    rec = {k: json.load(open(tmp_path / f"{k}.json")) for k in kinds}
    print("\n[brain-measured]", json.dumps({k: {"gpu_mix": v["gpu_mix"], "hbm_peak_gb": v["hbm_peak_gb"]}
                                            for k, v in rec.items()}))
    for k, v in rec.items():
        assert v["gpu_mix"].get("cu_probe", {}).get("probes", 0) >= 2, (k, v["gpu_mix"])
    metrics = {"job-worker-0:1": rec["compute"], "job-worker-1:2": rec["bandwidth"]}
    inv = NodeInventory(gpus=[GpuInfo(0, "gfx950", 256, 288.0)], cpus=16, host_mem_gb=512)
    plan = ResourcePlan(roles={"worker": RoleResource(2, Resource(gpu=1))}, bucket_mb=128.0)
    nxt = Planner().next_plan(JobFeatures(mode="allreduce", params=1e8, max_workers=2), inv, plan, metrics)
    assert nxt is not None
    print("[brain-measured] plan:", nxt.per_rank, nxt.reason)
    bw, cp = nxt.per_rank.get("job-worker-1:2", {}), nxt.per_rank.get("job-worker-0:1", {})
    assert 0 < bw.get("cu", 256) < 256, nxt.per_rank
    assert "cu" not in cp, nxt.per_rank
    assert rec["bandwidth"]["gpu_mix"]["cu_sensitivity"] < rec["compute"]["gpu_mix"]["cu_sensitivity"]
    for n, d in nxt.per_rank.items():
        assert d.get("hbm_gb") and d["hbm_gb"] < 288 * 0.85, nxt.per_rank
