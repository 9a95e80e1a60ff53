"""All-reduce policy from a measured size table (RCCL against the xGMI engine).

One pure function shared by the two places that decide:

* ``Communicator._probe_xgmi`` — every epoch, from the table its ranks just
  measured (each entry the MAX over ranks, so every rank derives the same
  policy from the same numbers);
* the Brain (``brain/planner.py``) — from the median of the tables every epoch
  of the same world size published, with a switching margin, pushed to the
  trainers as the runtime knob ``allreduce`` (they switch at one committed step).

Engine forms (csrc/kernels/xgmi.hip): ``oneshot`` (every rank reads every
peer's whole staged buffer: one barrier, latency-bound sizes), ``inplace``
(two-shot on a registered buffer: no staging copy) and ``staged`` (two-shot
through the workspace, for buffers too large to map).  The policy is

* ``oneshot_max_kb`` / ``oneshot_max_staged_kb``: the largest size at which
  one-shot still beats the registered / staged two-shot at every size below;
* ``xgmi_min_kb_inplace`` / ``xgmi_min_kb_staged``: the smallest size from
  which the engine (with the one-shot switch above) beats RCCL at every larger
  probed size (``0`` = from the smallest size on, ``None`` = never);
* ``bucket_floor_mb``: the smallest probed size whose best bus bandwidth is
  within ``knee`` of the best seen — gradient buckets below it waste link time.
"""
from __future__ import annotations

import math

INF = float("inf")


def _finite(x) -> bool:
    return x is not None and math.isfinite(x)


def busbw_gbs(size_kb: float, t_s: float, world: int) -> float:
    if not _finite(t_s) or t_s <= 0 or world <= 1:
        return 0.0
    return 2 * (world - 1) / world * size_kb * 1024 / t_s / 1e9


def _first_win(sizes, eng, rccl, margin):
    """Smallest size from which the engine wins at every larger size (0 = all, None = never)."""
    out = None
    for i in range(len(sizes) - 1, -1, -1):
        if _finite(eng[i]) and _finite(rccl[i]) and eng[i] < rccl[i] * (1.0 - margin):
            out = sizes[i]
        else:
            break
    if out is not None and out == sizes[0]:
        return 0
    return out


def _oneshot_max(sizes, oneshot, twoshot, margin):
    best = 0
    for s, o, t in zip(sizes, oneshot, twoshot):
        if _finite(o) and (not _finite(t) or o < t * (1.0 - margin)):
            best = s
        else:
            break
    return best


def decide(sizes_kb, rccl, inplace, staged, oneshot=None, world: int = 2, margin: float = 0.0,
           knee: float = 0.85) -> dict:
    """The all-reduce policy from per-size times in seconds (``inf`` = form unavailable)."""
    n = len(sizes_kb)
    oneshot = list(oneshot) if oneshot is not None else [INF] * n
    os_reg = _oneshot_max(sizes_kb, oneshot, inplace, margin)
    os_stg = _oneshot_max(sizes_kb, oneshot, staged, margin)
    reg = [oneshot[i] if sizes_kb[i] <= os_reg else inplace[i] for i in range(n)]
    stg = [oneshot[i] if sizes_kb[i] <= os_stg else staged[i] for i in range(n)]
    min_reg = _first_win(sizes_kb, reg, rccl, margin)
    min_stg = _first_win(sizes_kb, stg, rccl, margin)
    # bandwidth knee of the path each size would take (registered buffers: DDP's case)
    best = []
    for i in range(n):
        use_eng = min_reg is not None and sizes_kb[i] >= min_reg
        best.append(busbw_gbs(sizes_kb[i], reg[i] if use_eng else rccl[i], world))
    floor = None
    if best and max(best) > 0:
        top = max(best)
        floor = next(sizes_kb[i] for i in range(n) if best[i] >= knee * top) / 1024.0
    return {"oneshot_max_kb": os_reg, "oneshot_max_staged_kb": os_stg, "xgmi_min_kb_inplace": min_reg,
            "xgmi_min_kb_staged": min_stg, "bucket_floor_mb": floor,
            "busbw_gbs": [round(b, 1) for b in best]}


def median_table(probes: list[dict]) -> dict | None:
    """Per-size (lower) median over the published probe tables with the latest size grid."""
    probes = [p for p in probes if p and p.get("sizes_kb") and p.get("exact_everywhere")]
    if not probes:
        return None
    sizes = probes[-1]["sizes_kb"]
    probes = [p for p in probes if p["sizes_kb"] == sizes]
    out = {"sizes_kb": sizes, "n": len(probes)}
    for col in ("rccl_ms", "xgmi_inplace_ms", "xgmi_staged_ms", "xgmi_oneshot_ms"):
        vals = []
        for i in range(len(sizes)):
            xs = sorted(INF if (p.get(col) or [None] * len(sizes))[i] is None else float(p[col][i]) for p in probes)
            vals.append(xs[(len(xs) - 1) // 2])   # lower median: timing noise is one-sided (slower)
        out[col] = vals
    return out


def decide_from_probe(probe: dict, world: int, margin: float = 0.0) -> dict:
    def ms(col):
        return [INF if v is None else v / 1e3 for v in probe.get(col) or [None] * len(probe["sizes_kb"])]
    return decide(probe["sizes_kb"], ms("rccl_ms"), ms("xgmi_inplace_ms"), ms("xgmi_staged_ms"),
                  ms("xgmi_oneshot_ms"), world=world, margin=margin)
