"""Hardware inventory and telemetry for the Brain.

GPU inventory is read from the KFD topology in sysfs — no HIP context is
created, so the job master never initialises a GPU (and may later hand every
GPU to a worker).  Live telemetry (utilisation, HBM in use, power) comes from
``rocm-smi --json`` when available; per-step training metrics come from the
workers through the master's store (``metrics/<node>``).
"""
from __future__ import annotations

import glob
import json
import os
import shutil
import subprocess
from dataclasses import asdict, dataclass, field


@dataclass
class GpuInfo:
    index: int
    gfx: str = ""
    cus: int = 0
    mem_gb: float = 0.0
    numa: int = -1
    busy_pct: float | None = None
    mem_used_gb: float | None = None
    power_w: float | None = None


@dataclass
class NodeInventory:
    gpus: list[GpuInfo] = field(default_factory=list)
    cpus: int = 0
    host_mem_gb: float = 0.0

    def to_dict(self):
        return {"gpus": [asdict(g) for g in self.gpus], "cpus": self.cpus, "host_mem_gb": self.host_mem_gb}


def _read_props(path: str) -> dict:
    out = {}
    try:
        with open(path) as f:
            for line in f:
                parts = line.split()
                if len(parts) == 2:
                    try:
                        out[parts[0]] = int(parts[1])
                    except ValueError:
                        pass
    except OSError:
        pass
    return out


def kfd_gpus(root: str = "/sys/class/kfd/kfd/topology/nodes") -> list[GpuInfo]:
    gpus = []
    for node in sorted(glob.glob(os.path.join(root, "*")), key=lambda p: int(os.path.basename(p) or 0)):
        props = _read_props(os.path.join(node, "properties"))
        gfx = props.get("gfx_target_version", 0)
        if not gfx:
            continue  # CPU node
        cus = props.get("simd_count", 0) // max(1, props.get("simd_per_cu", 4))
        mem = 0
        for b in glob.glob(os.path.join(node, "mem_banks", "*", "properties")):
            mp = _read_props(b)
            mem = max(mem, mp.get("size_in_bytes", 0))
        g = GpuInfo(index=len(gpus), gfx=f"gfx{gfx // 10000}{(gfx // 100) % 100:x}{gfx % 100:x}", cus=cus,
                    mem_gb=mem / 2**30, numa=props.get("numa_node", -1) if "numa_node" in props else -1)
        gpus.append(g)
    return gpus


def rocm_smi_telemetry(gpus: list[GpuInfo]) -> list[GpuInfo]:
    exe = shutil.which("rocm-smi")
    if not exe:
        return gpus
    try:
        r = subprocess.run([exe, "--showuse", "--showmemuse", "--showpower", "--json"], capture_output=True,
                           text=True, timeout=10)
        data = json.loads(r.stdout or "{}")
    except Exception:
        return gpus
    for key, v in data.items():
        if not key.startswith("card"):
            continue
        try:
            i = int(key[4:])
        except ValueError:
            continue
        if i < len(gpus):
            for k, val in v.items():
                lk = k.lower()
                try:
                    fv = float(str(val).strip("%"))
                except ValueError:
                    continue
                if "gpu use" in lk:
                    gpus[i].busy_pct = fv
                elif "memory" in lk and ("use" in lk or "allocated" in lk):
                    gpus[i].mem_used_gb = fv / 100.0 * gpus[i].mem_gb
                elif "power" in lk:
                    gpus[i].power_w = fv
    return gpus


def host_inventory(telemetry: bool = False) -> NodeInventory:
    gpus = kfd_gpus()
    if telemetry:
        gpus = rocm_smi_telemetry(gpus)
    mem = 0.0
    try:
        mem = os.sysconf("SC_PAGE_SIZE") * os.sysconf("SC_PHYS_PAGES") / 2**30
    except (ValueError, OSError):
        pass
    return NodeInventory(gpus=gpus, cpus=os.cpu_count() or 1, host_mem_gb=mem)


# --------------------------------------------------------------------- rocprofv3
# Kernel classes by name: matrix-core work (hipBLASLt/Tensile GEMMs, our MFMA
# flash attention) vs. bandwidth-bound work (elementwise, norms, optimizer,
# copies, collectives).  A role whose GPU time is mostly bandwidth-bound keeps
# its throughput on a fraction of the 256 CUs — that is the Brain's CU signal.
_COMPUTE_PAT = ("Cijk_", "gemm", "attn_fwd", "attn_bwd_dq", "attn_bwd_dkdv", "mfma")
_COMM_PAT = ("ncclDevKernel", "rccl", "xgmi_")


def rocprof_kernel_profile(path: str) -> dict | None:
    """Summarise a ``rocprofv3 --kernel-trace --stats`` kernel-stats CSV.

    Accepts rocprofv3's own ``*_kernel_stats.csv`` (Name, TotalDurationNs, ...)
    and the trimmed copies under ``profiles/`` (kernel, total_ms, ...).  Returns
    ``{"total_ms", "compute_frac", "comm_frac", "memory_frac", "top": [...]}``.
    """
    import csv
    if not os.path.exists(path):
        return None
    with open(path) as f:
        lines = [ln for ln in f if not ln.startswith("#")]
    rows = list(csv.DictReader(lines))
    if not rows:
        return None
    items = []
    for r in rows:
        name = r.get("Name") or r.get("kernel") or ""
        if "TotalDurationNs" in r:
            ms = float(r["TotalDurationNs"]) / 1e6
        else:
            ms = float(r.get("total_ms") or 0.0)
        items.append((name, ms))
    total = sum(ms for _, ms in items) or 1.0
    comp = sum(ms for n, ms in items if any(p in n for p in _COMPUTE_PAT))
    comm = sum(ms for n, ms in items if any(p in n for p in _COMM_PAT))
    top = sorted(items, key=lambda x: -x[1])[:5]
    return {"total_ms": round(total, 3), "compute_frac": round(comp / total, 4), "comm_frac": round(comm / total, 4),
            "memory_frac": round(max(0.0, 1 - (comp + comm) / total), 4),
            "top": [{"kernel": n[:80], "ms": round(ms, 3)} for n, ms in top]}


def rocprof_rank_profiles(run_dir: str) -> dict[str, dict]:
    """Per-process kernel profiles a job left under ``<run_dir>/rocprof/<process>/*kernel_stats.csv``."""
    out = {}
    for p in glob.glob(os.path.join(run_dir, "rocprof", "*", "*kernel_stats.csv")):
        prof = rocprof_kernel_profile(p)
        if prof is not None:
            out[os.path.basename(os.path.dirname(p))] = prof
    return out


def collect_worker_metrics(kv, nodes: list[str]) -> dict[str, dict]:
    out = {}
    for n in nodes:
        m = kv.get(f"metrics/{n}")
        if m:
            out[n] = m
    return out
