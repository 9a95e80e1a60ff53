"""Unit tier: Brain periodic plans, bucket/interval sizing, and
the elastic shard dispatcher's requeue-on-death guarantees, on an in-process store."""
import datetime
import os
import socket

import torch.distributed as dist

from easydl_amd.api.spec import Resource, ResourcePlan, RoleResource
from easydl_amd.brain.collectors import GpuInfo, NodeInventory
from easydl_amd.brain.planner import JobFeatures, Planner, ckpt_interval, grad_bucket_mb, BrainConfig
from easydl_amd.master.dispatcher import ShardDispatcher
from easydl_amd.master.store import KV


ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _inv(n=8, busy=0.0):
    return NodeInventory(gpus=[GpuInfo(i, "gfx950", 256, 288.0, busy_pct=busy) for i in range(n)], cpus=128,
                         host_mem_gb=2048)


def _plan(workers=4, bucket=128.0):
    return ResourcePlan(roles={"worker": RoleResource(workers, Resource(gpu=1))}, bucket_mb=bucket)


def test_straggler_is_marked_for_eviction_after_a_full_window():
    p = Planner()
    feat = JobFeatures(params=8e9, max_workers=4)
    m = {f"w{i}": {"step_time": 1.0, "window": 20} for i in range(4)}
    m["w3"]["step_time"] = 1.6
    nxt = p.next_plan(feat, _inv(4, busy=90), _plan(), m)
    assert nxt is not None and nxt.per_rank["w3"]["evict"] is True
    assert "w0" not in nxt.per_rank
    m["w3"]["window"] = 5                      # not a full window yet: no eviction
    nxt = Planner().next_plan(feat, _inv(4, busy=90), _plan(), m)
    assert nxt is None or "w3" not in nxt.per_rank


def test_bucket_autotune_tries_neighbours_then_keeps_the_best():
    p = Planner()
    feat = JobFeatures(params=8e9, max_workers=4)
    times = {128.0: 1.00, 64.0: 1.10, 256.0: 0.95, 512.0: 0.97}
    plan = _plan(bucket=128.0)
    seen = []
    for _ in range(6):
        m = {f"w{i}": {"step_time": times[plan.bucket_mb], "window": 20} for i in range(4)}
        nxt = p.next_plan(feat, _inv(4, busy=90), plan, m)
        if nxt is None:
            break
        plan = nxt
        seen.append(plan.bucket_mb)
    assert plan.bucket_mb == 256.0, seen       # fastest measured size wins


def test_scale_up_into_free_gpus():
    nxt = Planner().next_plan(JobFeatures(params=1e9, max_workers=8), _inv(8), _plan(workers=4),
                              {"w0": {"step_time": 1.0}})
    assert nxt.roles["worker"].replicas == 8


def test_bucket_and_interval_sizing():
    assert grad_bucket_mb(8e9, 1) == 128.0
    b = grad_bucket_mb(8e9, 8)
    assert 64.0 <= b <= 512.0 and (int(b) & (int(b) - 1)) == 0     # power of two
    k1 = ckpt_interval(8e9, 1, 1.7, BrainConfig())
    k8 = ckpt_interval(8e9, 8, 1.7, BrainConfig())
    assert k1 > k8 >= 1                                               # sharding shortens the copy


def _kv():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return KV(dist.TCPStore("127.0.0.1", port, 1, True, timeout=datetime.timedelta(seconds=10)), "t")


def test_dispatcher_requeues_a_dead_workers_leases_exactly_once():
    kv = _kv()
    d = ShardDispatcher(kv, num_samples=1000, shard_size=100, epochs=1)
    a = [d.claim("A") for _ in range(3)]
    b = [d.claim("B") for _ in range(2)]
    d.complete(a[0])
    assert d.requeue_dead({"A"}) == [a[1], a[2]]      # completed shards are not requeued
    got = []
    while (s := d.claim("B")) is not None:
        got.append(s)
        d.complete(s)
    for s in b:
        d.complete(s)
    covered = sorted([a[0]] + b + got)
    assert covered == list(range(10)), covered         # every shard exactly once
    assert d.done() == 10


def test_rocprof_profile_drives_per_rank_cu_plan(tmp_path):
    """The Brain reads rocprofv3 kernel stats: a bandwidth-bound rank gets a CU share,
    a matrix-core-bound rank keeps the whole GPU."""
    from easydl_amd.brain.collectors import rocprof_kernel_profile
    ps = tmp_path / "ps_kernel_stats.csv"
    ps.write_text('"Name","Calls","TotalDurationNs","AverageNs","Percentage"\n'
                  '"void adamw_flat_kernel<float>",100,900000000,9000000,90\n'
                  '"Cijk_Ailk_Bljk_BBS_BH",10,100000000,10000000,10\n')
    prof = rocprof_kernel_profile(str(ps))
    assert prof["memory_frac"] == 0.9 and prof["compute_frac"] == 0.1
    train = rocprof_kernel_profile(os.path.join(ROOT, "profiles", "r01_bench_kernel_stats_latest.csv"))
    assert train["compute_frac"] > 0.85
    metrics = {"ps0": {"rocprof": prof}, "w0": {"step_time": 1.0, "rocprof": train}}
    nxt = Planner().next_plan(JobFeatures(mode="ps", params=3.3e8), _inv(8, busy=90), _plan(), metrics)
    assert nxt is not None and 0 < nxt.per_rank["ps0"]["cu"] < 256 and nxt.per_rank["ps0"]["cu"] % 8 == 0
    assert "cu" not in nxt.per_rank.get("w0", {})


def test_amdsmi_samples_give_link_rates_throttle_share_and_busy_by_hbm():
    from easydl_amd.brain.collectors import amdsmi_record, merge_amdsmi
    na = "N/A"

    def raw(rd, wr, ppt, acc):
        return {"average_gfx_activity": 97, "average_umc_activity": 41, "current_socket_power": na,
                "average_socket_power": 1350, "current_gfxclks": [2100, 2000, na, 2100, 2000, 2100, 2000, 2100],
                "ppt_residency_acc": ppt, "accumulation_counter": acc,
                "xgmi_read_data_acc": rd, "xgmi_write_data_acc": wr}

    a = amdsmi_record(raw([0] * 7 + [na], [0] * 8, 100, 1000), {"vram_used": 210 * 1024}, "0000:75:00.0")
    b = amdsmi_record(raw([50_000_000] * 7 + [na], [25_000_000] * 8, 350, 2000), {"vram_used": 210 * 1024},
                      "0000:75:00.0")
    a["t"], b["t"] = 10.0, 10.5
    gpus = [GpuInfo(0, "gfx950", 256, 288.0, bdf="0000:05:00.0"), GpuInfo(1, "gfx950", 256, 288.0,
                                                                          bdf="0000:75:00.0")]
    merge_amdsmi(gpus, [a], [b])
    g = gpus[1]                                          # matched by PCI address, not by order
    assert gpus[0].power_w is None and g.power_w == 1350 and g.busy_pct == 97 and g.umc_pct == 41
    assert g.xgmi_read_gbps[:7] == [100.0] * 7 and g.xgmi_read_gbps[7] is None   # 50 GB in 0.5 s
    assert g.xgmi_write_gbps == [50.0] * 8
    assert g.throttle_pct == 25.0 and abs(g.gfxclk_mhz - 2057.1) < 0.1
    assert g.mem_used_gb == 210.0 and g.is_busy()
    assert not GpuInfo(2, "gfx950", 256, 288.0, busy_pct=3, mem_used_gb=0.3).is_busy()
    # a GPU someone holds (HBM in use) is not "free" for a scale-up, even while idle: the
    # job's 4 workers hold GPUs 0-3, another process holds 6-7 -> room for 2 more workers
    inv = NodeInventory(gpus=[GpuInfo(i, "gfx950", 256, 288.0, busy_pct=0,
                                      mem_used_gb=0.2 if i in (4, 5) else 100.0) for i in range(8)],
                        cpus=128, host_mem_gb=2048)
    nxt = Planner().next_plan(JobFeatures(params=8e9, max_workers=8), inv, _plan(workers=4), {})
    assert nxt is not None and nxt.roles["worker"].replicas == 6


def _probe(epoch, world, rccl, inplace, exact=True):
    kb = [1024, 4096, 32768, 131072]
    return {"epoch": epoch, "world": world,
            "probe": {"sizes_kb": kb, "exact_everywhere": exact, "rccl_ms": rccl, "xgmi_inplace_ms": inplace,
                      "xgmi_staged_ms": [9.0] * 4, "xgmi_oneshot_ms": [0.02, None, None, None]}}


def test_brain_allreduce_policy_from_probe_median_and_bucket_knee():
    """The epochs' probe tables drive the all-reduce routing and the bucket floor:
    the policy follows the per-size MEDIAN (one noisy epoch does not flip it), a
    narrow engine win inside the margin stays with RCCL, and bucket sizes below the
    bandwidth knee are not tried."""
    p = Planner()
    feat = JobFeatures(params=8e9, max_workers=8)
    rccl = [0.040, 0.080, 0.400, 1.500]
    good = [0.045, 0.060, 0.300, 1.100]          # engine wins from 4 MB, one-shot at 1 MB
    plan = _plan(workers=8, bucket=32.0)
    m = {f"w{i}": {"step_time": 1.0, "window": 20} for i in range(8)}
    nxt = p.next_plan(feat, _inv(8, busy=90), plan, m, _probe(1, 8, rccl, good))
    assert nxt is not None and nxt.allreduce["dp"]["world"] == 8
    pol = nxt.allreduce["dp"]["policy"]
    assert pol["oneshot_max_kb"] == 1024 and pol["xgmi_min_kb_inplace"] == 0
    assert pol["xgmi_min_kb_staged"] is None and pol["oneshot_max_staged_kb"] == 1024
    assert pol["bucket_floor_mb"] == 32.0 and nxt.bucket_mb >= 32.0     # autotune goes on above the floor
    plan = nxt
    # one epoch where the engine looked slow everywhere: the median keeps the policy
    nxt = p.next_plan(feat, _inv(8, busy=90), plan, m, _probe(2, 8, rccl, [9.0] * 4))
    assert nxt is None or nxt.allreduce == plan.allreduce
    # narrow wins (< 3 %) at 4..128 MB: the per-epoch probe (no margin) would route them to
    # the engine, the Brain's policy keeps them on RCCL
    from easydl_amd.parallel.comm_policy import decide_from_probe
    narrow = [0.045, 0.079, 0.395, 1.49]
    assert decide_from_probe(_probe(0, 8, rccl, narrow)["probe"], 8)["xgmi_min_kb_inplace"] == 0
    p2 = Planner()
    nxt = p2.next_plan(feat, _inv(8, busy=90), _plan(workers=8), m, _probe(0, 8, rccl, narrow))
    assert nxt.allreduce["dp"]["policy"]["xgmi_min_kb_inplace"] is None, nxt.allreduce
    # inexact probes are never used
    p3 = Planner()
    assert p3.next_plan(feat, _inv(8, busy=90), _plan(workers=8), {}, _probe(0, 8, rccl, good, exact=False)) is None


def test_brain_bucket_floor_skips_sizes_below_the_knee():
    p = Planner()
    feat = JobFeatures(params=8e9, max_workers=8)
    # RCCL only: bus bandwidth keeps rising to 128 MB -> 32/64 MB buckets are below 85 %
    rccl = [0.040, 0.080, 0.700, 1.500]
    plan = _plan(workers=8, bucket=32.0)
    m = {f"w{i}": {"step_time": 1.0, "window": 20} for i in range(8)}
    nxt = p.next_plan(feat, _inv(8, busy=90), plan, m, _probe(1, 8, rccl, [9.0] * 4))
    assert nxt is not None and nxt.allreduce["dp"]["policy"]["xgmi_min_kb_inplace"] in (0, None)
    floor = nxt.allreduce["dp"]["policy"]["bucket_floor_mb"]
    assert floor == 128.0 and nxt.bucket_mb == 128.0, (floor, nxt.reason)


def test_plan_loop_writes_one_versioned_runtime_document(tmp_path):
    """master/planner.py: the plan's knobs (bucket, interval, all-reduce policy) go to
    plan/runtime/<v> before plan/version moves to v; the probe reaches the Brain."""
    import json
    from easydl_amd.api.spec import ElasticJob
    from easydl_amd.master.planner import PlanLoop

    kv = _kv()

    class Rdzv:
        target_nodes = 0

        def members(self):
            return [f"w{i}" for i in range(8)]

    class Events:
        def emit(self, *a, **k):
            pass

    class Master:
        pass

    master = Master()
    master.kv, master.rdzv, master.events, master.run_dir = kv, Rdzv(), Events(), str(tmp_path)

    class Brain:
        def __init__(self):
            self.p = Planner()

        def startup_plan(self, features):
            return _plan(workers=8, bucket=32.0)

        def next_plan(self, features, plan, metrics, comm=None):
            return self.p.next_plan(JobFeatures(params=8e9, max_workers=8), _inv(8, busy=90), plan, metrics, comm)

    job = ElasticJob.from_dict({"apiVersion": "elastic.easydl.org/v1alpha1", "kind": "ElasticJob",
                                "metadata": {"name": "t"}, "spec": {"worker": {"image": "x"}}})
    loop = PlanLoop(job, Brain(), period_s=0.001, user_wait_s=0.0)
    loop._features = {}
    loop.maybe_replan(master)                 # startup plan -> version 1
    assert kv.counter("plan/version") == 1
    assert kv.get("plan/runtime/1")["bucket_mb"] == 32.0
    for i in range(8):
        kv.set(f"metrics/w{i}", json.dumps({"step_time": 1.0, "window": 20}))
    kv.set("comm/probe/dp", json.dumps(_probe(1, 8, [0.040, 0.080, 0.400, 1.500], [0.045, 0.060, 0.300, 1.100])))
    kv.set("comm/probe/tp", json.dumps(_probe(1, 4, [0.040, 0.080, 0.400, 1.500], [0.09, 0.2, 0.9, 3.0])))
    import time
    time.sleep(0.01)
    loop.maybe_replan(master)
    assert kv.counter("plan/version") == 2
    doc = kv.get("plan/runtime/2")
    assert doc["allreduce"]["dp"]["world"] == 8 and doc["allreduce"]["dp"]["policy"]["oneshot_max_kb"] == 1024
    # the TP group (4 ranks) gets its own policy: its engine loses at every two-shot size
    assert doc["allreduce"]["tp"]["world"] == 4
    assert doc["allreduce"]["tp"]["policy"]["xgmi_min_kb_inplace"] is None
    assert json.loads(kv.get_str("jobresource"))["spec"]["allreduce"] == doc["allreduce"]


def test_startup_plan_sizes_snapshots_for_host_dram():
    """70B (TP) state: two full A/B copies (1.7 TB) exceed 1.5 TB of host DRAM, two lean
    copies (0.56 TB) fit; 8B fits in full."""
    inv = NodeInventory(gpus=[GpuInfo(i, "gfx950", 256, 288.0) for i in range(8)], cpus=128, host_mem_gb=1536)
    p70 = Planner().startup_plan(JobFeatures(params=70.6e9, activation_gb_per_rank=10, bytes_per_param_state=2),
                                 inv)
    assert "in-memory snapshots lean" in p70.reason, p70.reason
    p8 = Planner().startup_plan(JobFeatures(params=8.03e9), inv)
    assert "in-memory snapshots full" in p8.reason, p8.reason
    small = NodeInventory(gpus=inv.gpus, cpus=128, host_mem_gb=64)
    assert "in-memory snapshots off" in Planner().startup_plan(JobFeatures(params=8.03e9), small).reason
