"""Hardware inventory and telemetry for the Brain.

GPU inventory is read from the KFD topology in sysfs — no HIP context is
created, so the job master never initialises a GPU (and may later hand every
GPU to a worker).  Live telemetry comes from amd-smi: GFX and
memory-controller activity, HBM in use, socket power, clocks, power-throttle
residency and the per-link xGMI read/write byte counters, sampled twice so the
Brain sees link rates in GB/s.  amd-smi runs in a short-lived child process
(``python -m easydl_amd.brain.collectors --amdsmi``) so the master never opens
the device itself; ``rocm-smi --json`` is the fallback.  Per-step training
metrics come from the workers through the master's store (``metrics/<node>``).
"""
from __future__ import annotations

import glob
import json
import os
import shutil
import subprocess
import sys
import time
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
    bdf: str = ""
    umc_pct: float | None = None           # memory-controller activity
    gfxclk_mhz: float | None = None        # mean over XCDs
    throttle_pct: float | None = None      # share of the sample window spent power-throttled
    xgmi_read_gbps: list[float] | None = None   # per link, over the sample window
    xgmi_write_gbps: list[float] | None = None

    def is_busy(self) -> bool:
        """In use by someone: computing, or holding more HBM than an idle context does."""
        return (self.busy_pct or 0) > 50 or (self.mem_used_gb or 0) > 8.0


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
        loc = props.get("location_id", 0)     # (bus << 8) | (device << 3) | function
        bdf = f"{props.get('domain', 0):04x}:{loc >> 8:02x}:{(loc >> 3) & 31:02x}.{loc & 7:x}" if loc else ""
        g = GpuInfo(index=len(gpus), gfx=f"gfx{gfx // 10000}{(gfx // 100) % 100:x}{gfx % 100:x}", cus=cus,
                    mem_gb=mem / 2**30, numa=props.get("numa_node", -1) if "numa_node" in props else -1, bdf=bdf)
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


# ---------------------------------------------------------------------- amd-smi
def _num(v):
    return None if v in (None, "N/A") or isinstance(v, str) else v


def amdsmi_record(metrics: dict, vram: dict | None, bdf: str = "") -> dict:
    """One GPU's raw amd-smi sample, normalised ("N/A" -> None; vram in MB, xGMI in KB)."""
    def links(key):
        v = metrics.get(key)
        return [None if _num(x) is None else int(x) for x in v] if isinstance(v, list) else None

    clks = [c for c in metrics.get("current_gfxclks") or [] if _num(c)] \
        if isinstance(metrics.get("current_gfxclks"), list) else []
    power = _num(metrics.get("current_socket_power"))
    if power is None:
        power = _num(metrics.get("average_socket_power"))
    return {"bdf": bdf, "t": time.monotonic(),
            "busy_pct": _num(metrics.get("average_gfx_activity")),
            "umc_pct": _num(metrics.get("average_umc_activity")),
            "power_w": power,
            "gfxclk_mhz": sum(clks) / len(clks) if clks else None,
            "ppt_acc": _num(metrics.get("ppt_residency_acc")),
            "acc": _num(metrics.get("accumulation_counter")),
            "vram_used_mb": _num((vram or {}).get("vram_used")),
            "xgmi_read_kb": links("xgmi_read_data_acc"),
            "xgmi_write_kb": links("xgmi_write_data_acc")}


def amdsmi_sample() -> list[dict]:
    """Read every GPU through the amdsmi Python binding (call it in a child process)."""
    import amdsmi
    amdsmi.amdsmi_init()
    try:
        out = []
        for h in amdsmi.amdsmi_get_processor_handles():
            try:
                bdf = amdsmi.amdsmi_get_gpu_device_bdf(h)
            except Exception:
                bdf = ""
            try:
                vram = amdsmi.amdsmi_get_gpu_vram_usage(h)
            except Exception:
                vram = None
            out.append(amdsmi_record(amdsmi.amdsmi_get_gpu_metrics_info(h), vram, bdf))
        return out
    finally:
        amdsmi.amdsmi_shut_down()


def _rate(a, b, dt):
    if a is None or b is None or dt <= 0:
        return None
    return [round((y - x) * 1e3 / dt / 1e9, 3) if x is not None and y is not None and y >= x else None
            for x, y in zip(a, b)]


def merge_amdsmi(gpus: list[GpuInfo], first: list[dict], second: list[dict] | None = None) -> list[GpuInfo]:
    """Fill ``gpus`` from one or two amd-smi samples.  Matched by PCI address when the
    KFD topology gave one, else by order.  Two samples give xGMI link rates and the
    power-throttle share of the window."""
    by_bdf = {g.bdf.lower(): g for g in gpus if g.bdf}
    for i, cur in enumerate(second or first):
        g = by_bdf.get((cur.get("bdf") or "").lower()) or (gpus[i] if i < len(gpus) else None)
        if g is None:
            continue
        g.busy_pct = cur["busy_pct"] if cur["busy_pct"] is not None else g.busy_pct
        if cur["power_w"] is not None:
            g.power_w = cur["power_w"]
        g.umc_pct, g.gfxclk_mhz = cur["umc_pct"], cur["gfxclk_mhz"]
        if cur["vram_used_mb"] is not None:
            g.mem_used_gb = cur["vram_used_mb"] / 1024.0
        if second is not None and i < len(first):
            prev = first[i]
            dt = cur["t"] - prev["t"]
            g.xgmi_read_gbps = _rate(prev["xgmi_read_kb"], cur["xgmi_read_kb"], dt)
            g.xgmi_write_gbps = _rate(prev["xgmi_write_kb"], cur["xgmi_write_kb"], dt)
            if None not in (prev["ppt_acc"], cur["ppt_acc"], prev["acc"], cur["acc"]) and cur["acc"] > prev["acc"]:
                g.throttle_pct = round(100.0 * (cur["ppt_acc"] - prev["ppt_acc"]) / (cur["acc"] - prev["acc"]), 1)
    return gpus


def amdsmi_telemetry(gpus: list[GpuInfo], window_s: float = 0.5) -> list[GpuInfo] | None:
    """Two amd-smi samples ``window_s`` apart, taken by a child process.  None when
    amd-smi is unavailable (no driver, no binding)."""
    try:
        r = subprocess.run([sys.executable, "-m", "easydl_amd.brain.collectors", "--amdsmi", str(window_s)],
                           capture_output=True, text=True, timeout=20 + window_s,
                           cwd=os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
        data = json.loads(r.stdout.strip().splitlines()[-1]) if r.returncode == 0 and r.stdout.strip() else None
    except Exception:
        return None
    if not data or not data.get("first"):
        return None
    return merge_amdsmi(gpus, data["first"], data.get("second"))


def host_inventory(telemetry: bool = False) -> NodeInventory:
    gpus = kfd_gpus()
    if telemetry:
        gpus = amdsmi_telemetry(gpus) or rocm_smi_telemetry(gpus)
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


def _main(argv=None):
    import argparse
    ap = argparse.ArgumentParser()
    ap.add_argument("--amdsmi", type=float, metavar="WINDOW_S", help="two amd-smi samples WINDOW_S apart, as JSON")
    a = ap.parse_args(argv)
    if a.amdsmi is not None:
        first = amdsmi_sample()
        second = None
        if a.amdsmi > 0:
            time.sleep(a.amdsmi)
            second = amdsmi_sample()
        print(json.dumps({"first": first, "second": second}), flush=True)
    else:
        print(json.dumps(host_inventory(True).to_dict()), flush=True)


if __name__ == "__main__":
    _main()
