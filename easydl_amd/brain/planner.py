"""Brain planners: startup resources and periodic re-plans
(reference README.md:13,19-23 "generate resources plans ... monitor the
performance of a training job and dynamically adjust the resources";
docs/design/elastic-training-operator.md:106-112).

The reference publishes no algorithm; this is
easydl_amd's, specialised for one 8x MI355X node:

Startup plan (from job features + node inventory)
* all-reduce jobs: one worker per free GPU (bounded by min/max workers);
  memory check — 16 B/param of training state + activations must fit the
  288 GB HBM of each rank, otherwise the plan refuses with a reason;
* PS jobs: PS count from the fp32 parameter+optimizer bytes (one PS per
  ``ps_shard_gb``) and the rest of the GPUs as workers; PS ranks get a CU
  share (their update kernel is HBM-bound and needs few CUs) — realised by the
  operator as CU-masked streams (``EDL_CU_MASK``) and an HBM cap;
* gradient bucket size for xGMI: large enough that each of the 7 links moves
  >= ~8 MiB per collective step, capped so ~4+ buckets overlap backward;
* in-memory checkpoint interval so snapshot D2H cost stays < 5 % of step time.

Periodic plan (from per-rank step metrics)
* straggler eviction: a rank slower than ``straggler_ratio`` x median for a
  full window is replaced (resource_updation re-creates it);
* bucket-size autotune: try neighbouring sizes window by window, keep the
  fastest measured step time — only over sizes at or above the all-reduce
  bandwidth knee the probes measured;
* all-reduce routing: every epoch's communicator times RCCL against the xGMI
  engine's forms at 256 KB..128 MB and publishes the table (``comm/probe/dp``,
  ``comm/probe/tp``: DP gradient buckets and TP activations get separate policies);
  the Brain takes the per-size median over the epochs of the same world size and
  re-derives the policy (one-shot switch sizes, the size from which the engine
  beats RCCL, with a margin in RCCL's favour) — a runtime knob the trainers switch
  to at one committed step (parallel/comm_policy.py);
* scale up to free GPUs when the job asked for more workers than it got.
"""
from __future__ import annotations

import math
import os
import statistics
from dataclasses import dataclass

from easydl_amd.api.spec import Resource, ResourcePlan, RoleResource
from easydl_amd.brain.collectors import NodeInventory

HBM_GB = 288.0
XGMI_LINKS = 7


@dataclass
class JobFeatures:
    """What the trainer master extracts from the job (reference :106 "extracts features")."""
    mode: str = "allreduce"
    params: float = 0.0              # parameter count
    bytes_per_param_state: float = 16.0
    tokens_per_step_per_rank: float = 8192.0
    activation_gb_per_rank: float = 40.0
    step_time_s: float | None = None
    min_workers: int = 1
    max_workers: int = 8
    host_mem_gb: float | None = None

    @classmethod
    def from_dict(cls, d: dict) -> "JobFeatures":
        f = cls()
        for k, v in (d or {}).items():
            if hasattr(f, k):
                setattr(f, k, type(getattr(f, k))(v) if getattr(f, k) is not None and v is not None else v)
        return f


@dataclass
class BrainConfig:
    ps_shard_gb: float = 8.0
    ps_cu: int = 64
    straggler_ratio: float = 1.3
    window: int = 20
    bucket_choices: tuple = (32.0, 64.0, 128.0, 256.0, 512.0)
    ckpt_overhead: float = 0.05
    pcie_gbps: float = 50.0
    snapshot_host_fraction: float = 0.8   # host DRAM the in-memory snapshot slots may take
    comm_margin: float = 0.03       # the engine must beat RCCL by this share to take a size
    comm_history: int = 8           # probe tables kept per world size
    # a host-CPU parameter server busier than this share of its window gets twice the cores
    ps_busy_high: float = float(os.environ.get("EDL_BRAIN_PS_BUSY_HIGH", 0.75))
    ps_cpu_max: int = int(os.environ.get("EDL_BRAIN_PS_CPU_MAX", 16))


def grad_bucket_mb(params: float, world: int, grad_bytes: int = 2) -> float:
    """Bucket size for an xGMI mesh: >= 8 MiB per link-step, >= 4 buckets per backward."""
    if world <= 1:
        return 128.0
    total_mb = params * grad_bytes / 2**20
    link_floor = 8.0 * XGMI_LINKS * world / max(1, world - 1)   # MiB so each ring step moves >= 8 MiB
    cap = max(link_floor, total_mb / 4)
    choice = 2 ** math.ceil(math.log2(max(link_floor, min(cap, 256.0))))
    return float(min(512.0, choice))


def ckpt_interval(params: float, world: int, step_time_s: float | None, cfg: BrainConfig) -> int:
    """Steps between in-memory snapshots so the sharded D2H stays under cfg.ckpt_overhead."""
    state_gb = params * 14 / 2**30            # bf16 params + fp32 master/m/v (grads excluded)
    per_rank_gb = state_gb / max(1, world)
    copy_s = per_rank_gb / cfg.pcie_gbps
    st = step_time_s or 1.0
    return max(1, int(math.ceil(copy_s / (cfg.ckpt_overhead * st))))


def snapshot_mode(feat: JobFeatures, inv: NodeInventory, cfg: BrainConfig) -> str | None:
    """Host-DRAM check for the node's A/B snapshot slots: DP ranks shard
    the replicated state, TP ranks each hold a unique shard, so the node always holds
    two copies of the whole state: 12 B/param (fp32 master + Adam moments), or 4 B/param
    for lean (master-only) snapshots.  The trainers' CheckpointManager makes the same
    decision from the live MemAvailable; this puts it in the plan up front."""
    host = inv.host_mem_gb or feat.host_mem_gb
    if not host or not feat.params or feat.mode == "ps":
        return None
    budget = cfg.snapshot_host_fraction * host
    full, lean = 2 * 12 * feat.params / 2**30, 2 * 4 * feat.params / 2**30
    if full <= budget:
        return f"full ({full:.0f} of {host:.0f} GB host DRAM)"
    if lean <= budget:
        return f"lean: moments dropped ({lean:.0f} GB; full needs {full:.0f} of {host:.0f} GB)"
    return f"off ({lean:.0f} GB even lean > {budget:.0f} GB)"


class Planner:
    def __init__(self, cfg: BrainConfig | None = None):
        self.cfg = cfg or BrainConfig()
        self._tune: dict = {}
        self._probes: dict[tuple, dict[int, dict]] = {}   # (group, world) -> epoch -> probe table

    # ------------------------------------------------------------------ startup
    def startup_plan(self, feat: JobFeatures, inv: NodeInventory) -> ResourcePlan:
        ngpu = len(inv.gpus)
        plan = ResourcePlan(reason="startup")
        if feat.mode == "ps":
            state_gb = feat.params * 12 / 2**30  # fp32 param + m + v on the PS
            n_ps = max(1, math.ceil(state_gb / self.cfg.ps_shard_gb)) if feat.params else 1
            if ngpu:
                # dense pushes: every worker step writes the whole gradient (4 B/param) into the
                # PS's HBM over xGMI -> one PS per 4 GPUs keeps the PS inbound links and its
                # HBM update below the workers' step rate (BERT-large: 2 PS + 6 workers)
                if feat.params * 4 > 1e9:
                    n_ps = max(n_ps, ngpu // 4)
                n_ps = min(n_ps, max(1, ngpu // 4))
                n_workers = max(feat.min_workers, min(feat.max_workers, ngpu - n_ps))
                ps_res = Resource(cpu=4, memory=max(4096, state_gb / n_ps * 1024 * 2), gpu=1, cu=self.cfg.ps_cu,
                                  hbm_gb=min(HBM_GB, state_gb / n_ps * 2 + 8))
                w_res = Resource(cpu=max(1, inv.cpus // max(1, ngpu)), gpu=1)
            else:
                n_workers = max(feat.min_workers, min(feat.max_workers, max(1, (inv.cpus - n_ps) // 2)))
                ps_res = Resource(cpu=1, memory=1024, gpu=0)
                w_res = Resource(cpu=1, memory=1024, gpu=0)
            plan.roles["parameter_server"] = RoleResource(n_ps, ps_res)
            plan.roles["worker"] = RoleResource(n_workers, w_res)
            plan.roles["evaluator"] = RoleResource(0, Resource(cpu=1, gpu=0))
            plan.reason = f"ps: {n_ps} PS for {state_gb:.1f} GB of state, {n_workers} workers"
        else:
            need = feat.params * feat.bytes_per_param_state / 2**30 + feat.activation_gb_per_rank
            if ngpu and need > HBM_GB:
                plan.reason = f"refused: {need:.0f} GB per rank exceeds {HBM_GB:.0f} GB HBM (use TP)"
                plan.roles["worker"] = RoleResource(0, Resource(gpu=1))
                return plan
            n = min(feat.max_workers, ngpu) if ngpu else feat.min_workers
            n = max(feat.min_workers, n)
            cpus = max(1, inv.cpus // max(1, n))
            plan.roles["worker"] = RoleResource(n, Resource(cpu=cpus, gpu=1 if ngpu else 0))
            plan.reason = f"allreduce: {n} workers x 1 GPU, {need:.0f} GB/rank"
        world = plan.roles["worker"].replicas
        plan.bucket_mb = grad_bucket_mb(feat.params, world)
        plan.ckpt_interval = ckpt_interval(feat.params, world, feat.step_time_s, self.cfg)
        mode = snapshot_mode(feat, inv, self.cfg)
        if mode is not None:
            plan.reason += f"; in-memory snapshots {mode}"
        return plan

    @staticmethod
    def cu_for_sensitivity(s: float | None, total_cus: int = 256, tol: float = 0.05,
                           floor: float = 0.25) -> int | None:
        """Fewest CUs that keep a rank within ``tol`` of its full-chip speed, from its MEASURED
        CU sensitivity ``s`` (utils/kmix.py: the share of its GPU time that scales with CUs).
        With ``t(c) = t_C * (1 + s * (C / c - 1))`` the slowdown stays <= tol for
        ``c >= C * s / (s + tol)``; never below ``floor`` of the chip (~1/4 of the CUs saturate
        HBM with 16-byte accesses).  None (keep every CU) when that is >= 90 % of the chip."""
        if s is None:
            return None
        frac = max(floor, s / (s + tol)) if s > 0 else floor
        if frac >= 0.9:
            return None
        return int(math.ceil(total_cus * frac / 8)) * 8   # whole CUs per XCD

    @classmethod
    def cu_for_profile(cls, prof: dict, total_cus: int = 256) -> int | None:
        """CUs for a rank from a measured profile: its probed CU sensitivity (``cu_sensitivity``,
        live) when present; else a rocprofv3 kernel profile's MFMA share (kernel names:
        matrix-core heavy ranks keep every CU, bandwidth-bound ranks need only enough CUs to
        saturate HBM, scaled by their compute share).  A phase split alone (which block
        launched the kernels, utils/kmix.py) is a label, not a measurement: no CU plan."""
        if prof.get("cu_sensitivity") is not None:
            return cls.cu_for_sensitivity(float(prof["cu_sensitivity"]), total_cus)
        if "top" not in prof and prof.get("source") != "rocprofv3":
            return None
        comp = prof.get("compute_frac", 1.0)
        if comp >= 0.5:
            return None
        frac = max(0.25, min(1.0, 0.25 + comp))
        return int(round(total_cus * frac / 8)) * 8   # whole CUs per XCD

    @staticmethod
    def sensitivity_from_telemetry(g) -> float | None:
        """A GPU that runs ONE rank and has no probe yet: amd-smi's memory-controller activity
        over its graphics activity (``average_umc_activity`` / ``average_gfx_activity``) --
        bandwidth-bound kernels keep the memory controllers busy for most of the GPU's busy
        time, matrix-core kernels for a fraction of it.  Coarse: used only at the extremes."""
        busy, umc = getattr(g, "busy_pct", None), getattr(g, "umc_pct", None)
        if busy is None or umc is None or busy < 30:
            return None
        share = umc / busy
        if share >= 0.7:
            return 0.05          # bandwidth-bound
        if share <= 0.35:
            return 1.0           # matrix-core bound
        return None

    @staticmethod
    def hbm_for_rank(m: dict, margin: float = 1.15, slack_gb: float = 2.0) -> float | None:
        """Per-rank HBM cap from what the rank's allocator really held at its peak
        (``hbm_peak_gb``, trainer metrics): peak x margin + slack, when that is clearly below
        the cap it runs under now (its current plan, else the whole GPU) -- the headroom goes
        back to the GPU's other tenants (a PS, an evaluator, a hot standby)."""
        peak = m.get("hbm_peak_gb")
        if not peak:
            return None
        want = float(math.ceil(peak * margin + slack_gb))
        cap = m.get("hbm_cap_gb") or m.get("hbm_total_gb") or HBM_GB
        return want if want < 0.85 * cap else None

    # ------------------------------------------------------------------ communication
    GROUPS = ("dp", "tp")

    @staticmethod
    def _by_group(comm: dict | None) -> dict:
        """``{"dp": doc, "tp": doc}`` (a single ``{"world", "epoch", "probe"}`` doc is DP's)."""
        if not comm:
            return {}
        if "probe" in comm:
            return {"dp": comm}
        return {g: d for g, d in comm.items() if isinstance(d, dict) and d.get("probe")}

    def observe_probe(self, comm: dict | None) -> None:
        """Keep the epochs' published all-reduce probe tables, per (group, world size)."""
        for group, doc in self._by_group(comm).items():
            world, epoch = int(doc.get("world", 0)), int(doc.get("epoch", 0))
            hist = self._probes.setdefault((group, world), {})
            hist[epoch] = doc["probe"]
            for e in sorted(hist)[:-self.cfg.comm_history]:
                del hist[e]

    def allreduce_plan(self, world: int, group: str = "dp") -> dict | None:
        """The all-reduce policy of a ``group`` of ``world`` ranks from the median of its probe tables."""
        from easydl_amd.parallel import comm_policy
        hist = self._probes.get((group, world), {})
        tab = comm_policy.median_table([hist[e] for e in sorted(hist)])
        if tab is None:
            return None
        pol = comm_policy.decide_from_probe(tab, world, margin=self.cfg.comm_margin)
        return {"world": world, "epochs": tab["n"], "policy": pol}

    # ------------------------------------------------------------------ periodic
    def next_plan(self, feat: JobFeatures, inv: NodeInventory, current: ResourcePlan,
                  metrics: dict[str, dict], comm: dict | None = None) -> ResourcePlan | None:
        """Return a changed plan, or None to keep the current one.  ``comm``: the latest
        published all-reduce probes per communicator group (``comm/probe/dp``,
        ``comm/probe/tp``), if any.  The plan's ``allreduce`` holds one policy per group:
        the DP gradient buckets and the TP activation all-reduces each get their own."""
        import copy
        plan = copy.deepcopy(current)
        changed = []
        self.observe_probe(comm)
        floor = None
        keys = ("oneshot_max_kb", "oneshot_max_staged_kb", "xgmi_min_kb_inplace", "xgmi_min_kb_staged")
        for group, doc in self._by_group(comm).items():
            ar = self.allreduce_plan(int(doc["world"]), group)
            if ar is None:
                continue
            if group == "dp":
                floor = ar["policy"].get("bucket_floor_mb")
            old = (current.allreduce or {}).get(group) or {}
            if (old.get("world") != ar["world"]
                    or any((old.get("policy") or {}).get(k) != ar["policy"].get(k) for k in keys)):
                plan.allreduce = dict(plan.allreduce or {}, **{group: ar})
                p = ar["policy"]
                changed.append(f"{group} all-reduce policy (world {ar['world']}, {ar['epochs']} probes): engine "
                               f"from {p['xgmi_min_kb_inplace']} KB in place / {p['xgmi_min_kb_staged']} KB staged, "
                               f"one-shot <= {p['oneshot_max_kb']} KB")
        times = {n: m.get("step_time") for n, m in metrics.items() if m.get("step_time")}
        if len(times) >= 2:
            med = statistics.median(times.values())
            for n, t in times.items():
                m = metrics[n]
                if t > self.cfg.straggler_ratio * med and m.get("window", 0) >= self.cfg.window:
                    plan.per_rank.setdefault(n, {})["evict"] = True
                    changed.append(f"straggler {n} ({t:.3f}s vs median {med:.3f}s)")
        # bucket autotune over windows of identical membership
        if times:
            st = statistics.median(times.values())
            t = self._tune
            cur = plan.bucket_mb or 128.0
            t.setdefault("results", {})
            t["results"][cur] = min(st, t["results"].get(cur, float("inf")))
            choices = list(self.cfg.bucket_choices)
            if floor:
                # buckets below the measured bandwidth knee leave link time on the table
                choices = [c for c in choices if c >= floor] or choices[-1:]
            # hill-climb around the best size measured so far: try its untried neighbours,
            # settle on it once both have been measured
            allowed = {c: v for c, v in t["results"].items() if c in choices}
            best = min(allowed, key=allowed.get) if allowed else None
            if best is None and floor:
                plan.bucket_mb = choices[0]
                changed.append(f"bucket {cur} MB is below the all-reduce bandwidth knee ({floor} MB): "
                               f"{choices[0]} MB")
            elif best is not None:
                i = choices.index(best)
                untried = [c for c in (choices[i - 1] if i > 0 else None, choices[i + 1] if i + 1 < len(choices)
                                       else None) if c is not None and c not in t["results"]]
                if untried:
                    if untried[0] != cur:
                        plan.bucket_mb = untried[0]
                        changed.append(f"bucket autotune: try {untried[0]} MB (best so far {best} MB)")
                elif best != cur:
                    plan.bucket_mb = best
                    changed.append(f"bucket autotune: best {best} MB")
        # per-rank CU and HBM plans from measurements (no role or phase labels): the rank's probed
        # CU sensitivity (metrics[n]["gpu_mix"]["cu_sensitivity"], utils/kmix.py), a rocprofv3
        # kernel profile (metrics[n]["rocprof"]), or -- a GPU with one rank and no probe -- its
        # amd-smi memory-controller vs graphics activity; the HBM cap from the rank's allocator
        # peak.  A rank is re-planned only when the plan differs from what it runs under now.
        per_gpu: dict = {}
        for n, m in metrics.items():
            if m.get("gpu") is not None and m.get("device", "cuda") == "cuda":
                per_gpu.setdefault(int(m["gpu"]), []).append(n)
        # ranks sharing a GPU: the most CU-sensitive one keeps every CU (a slice is only worth
        # giving to the co-tenants that lose least from it)
        keep_all = set()
        for g, names in per_gpu.items():
            probed = [(float((metrics[n].get("gpu_mix") or {}).get("cu_sensitivity")), n) for n in names
                      if (metrics[n].get("gpu_mix") or {}).get("cu_sensitivity") is not None]
            if len(probed) >= 2:
                keep_all.add(max(probed)[1])
        for n, m in metrics.items():
            prof = m.get("rocprof") or m.get("gpu_mix")
            cu, src = None, None
            if n in keep_all:
                prof = None         # keeps every CU; its HBM cap is still planned below
            if prof and (m.get("device", "cuda") == "cuda" or m.get("rocprof")):
                cu = self.cu_for_profile(prof)
                if prof.get("cu_sensitivity") is not None:
                    src = f"CU sensitivity {prof['cu_sensitivity']:.2f} measured on half the CUs"
                elif m.get("rocprof"):
                    src = f"rocprofv3: {100 * prof.get('memory_frac', 0):.0f}% of GPU time bandwidth-bound"
            has_probe = bool(prof and prof.get("cu_sensitivity") is not None)
            g = m.get("gpu")
            if (cu is None and not has_probe and not m.get("rocprof") and g is not None
                    and len(per_gpu.get(int(g), [])) == 1 and int(g) < len(inv.gpus)):
                s_tel = self.sensitivity_from_telemetry(inv.gpus[int(g)])
                cu = self.cu_for_sensitivity(s_tel)
                if cu is not None:
                    gi = inv.gpus[int(g)]
                    src = f"amd-smi: umc {gi.umc_pct:.0f}% of gfx {gi.busy_pct:.0f}%"
            if cu is not None and cu != m.get("cu"):
                plan.per_rank.setdefault(n, {})["cu"] = cu
                changed.append(f"{n}: {cu} CUs ({src})")
            hbm = self.hbm_for_rank(m) if m.get("device", "cuda") == "cuda" else None
            if hbm is not None and hbm != m.get("hbm_cap_gb"):
                plan.per_rank.setdefault(n, {})["hbm_gb"] = hbm
                changed.append(f"{n}: HBM cap {hbm:.0f} GB (peak {m['hbm_peak_gb']:.1f} GB)")
            # a parameter server on host CPUs that is busy most of the time: more cores
            if m.get("role") == "ps" and m.get("device") == "cpu" and m.get("busy_frac", 0) > self.cfg.ps_busy_high:
                cpu = int(m.get("cpu") or 1)
                want = min(self.cfg.ps_cpu_max, 2 * cpu)
                if want > cpu:
                    plan.per_rank.setdefault(n, {})["cpu"] = want
                    changed.append(f"{n}: {want} CPUs (busy {100 * m['busy_frac']:.0f}% on {cpu})")
        # grow into free GPUs
        wr = plan.roles.get("worker")
        if wr is not None and feat.mode != "ps":
            busy = sum(1 for g in inv.gpus if g.is_busy())
            free = len(inv.gpus) - max(busy, wr.replicas)
            if free > 0 and wr.replicas < feat.max_workers:
                wr.replicas = min(feat.max_workers, wr.replicas + free)
                changed.append(f"scale up to {wr.replicas} workers")
        if not changed:
            return None
        plan.reason = "; ".join(changed)
        return plan
