"""Hand the training state's HBM from a dying worker to the hot standby on its GPU.

Why (round 4 no-survivor restore, ``profiles/r04_ttr_n1_restore.md``): a replacement on the
GPU of a killed Llama-3-8B worker spent 5.4 s of its 10 s time-to-recover inside
``hipMalloc`` of its 128 GB of flat parameters, gradients and AdamW state.  The dead
process's 210 GB are released by the driver only after its teardown, and new allocations
wait until it has reclaimed them (``docs/design_notes.md``, "TTR is dominated by the
driver").

How: every worker exports its persistent state tensors as IPC handles into the job store
(``vram/gpu<k>``).  The parked standby imports them while the worker is still alive.  The
imports keep the physical memory referenced, so when the worker dies those 128 GB are never
released or reclaimed.  At takeover the standby's ``FlatParams`` / ``FlatAdamW`` build on
the imported tensors (``take``) instead of allocating.  The restore then overwrites them
from the shm snapshot as before: the dead worker may have died in the middle of an update.

Constraint: ``hipIpcOpenMemHandle`` hangs on allocations of 2 GiB or more on this stack
(``profiles/r03_ipc_size_probe2.txt``), so with hand-over on, flat groups are capped at
960 MiB of bf16 and their fp32 master / moments stay under 2 GiB (``FlatParams``).  A larger
tensor is simply not exported and is allocated as usual at takeover.

``EDL_VRAM_HANDOFF=1`` turns it on.  The local operator sets it for workers and standbys
when the job runs hot standbys.
"""
from __future__ import annotations

import json
import logging
import os
import time

import torch

log = logging.getLogger(__name__)

IPC_MAX_BYTES = 2040 << 20       # largest allocation hipIpcOpenMemHandle maps here
GROUP_MAX_MB = 960               # flat-group cap (bf16) under hand-over: fp32 state < 2 GiB

_ADOPTED: dict[str, torch.Tensor] = {}
TAKEN: dict[str, int] = {}       # name -> data_ptr of every adopted tensor a buffer was built on
STATS = {"exported": 0, "adopted": 0, "adopted_bytes": 0}
FAILED: list[str] = []           # names the last publish could not export


def enabled() -> bool:
    return os.environ.get("EDL_VRAM_HANDOFF", "0") == "1"


def key(slot: str) -> str:
    """Store key of one worker slot's export (``worker<index>``: the slot a replacement takes over)."""
    return f"vram/{slot}"


def _block_bytes(t: torch.Tensor) -> int:
    return t.untyped_storage().nbytes()


def _segments(device) -> list[tuple[int, int]]:
    """(base address, bytes) of every caching-allocator segment on ``device``, sorted."""
    idx = torch.device(device).index
    return sorted((int(sg["address"]), int(sg["total_size"])) for sg in torch.cuda.memory_snapshot()
                  if sg.get("device") == idx)


def _segment_bytes(segs: list[tuple[int, int]], ptr: int) -> int:
    """Size of the segment holding ``ptr`` (0: not a caching-allocator allocation, e.g. imported)."""
    import bisect
    i = bisect.bisect_right(segs, (ptr, float("inf"))) - 1
    if i >= 0 and segs[i][0] <= ptr < segs[i][0] + segs[i][1]:
        return segs[i][1]
    return 0


def publish(kv, slot: str, owner: str, tensors: dict[str, torch.Tensor]) -> int:
    """Export ``tensors`` (name -> CUDA tensor owning its whole allocation) for the standby.
    An IPC handle maps the tensor's whole caching-allocator segment: a tensor that sits in a
    segment of IPC_MAX_BYTES or more (e.g. a buffer allocated after a step, carved out of a
    cached activation segment) is not exported -- the standby's open would hang."""
    from easydl_amd.ps.ipc import export_tensor
    descs = {}
    STATS["export_failed"] = 0
    STATS.pop("export_error", None)
    FAILED.clear()
    devs = {t.device for t in tensors.values() if t is not None and t.is_cuda}
    segs = {d: _segments(d) for d in devs}
    for name, t in tensors.items():
        if t is None or not t.is_cuda or _block_bytes(t) > IPC_MAX_BYTES:
            continue
        if _segment_bytes(segs[t.device], t.data_ptr()) > IPC_MAX_BYTES:
            STATS["export_failed"] += 1
            STATS["export_error"] = f"{name}: in a segment of 2 GiB or more"
            FAILED.append(name)
            continue
        try:
            descs[name] = export_tensor(t)
        except RuntimeError as e:   # e.g. a tensor this process itself imported (an adopted buffer)
            log.debug("vram: %s not exportable: %s", name, e)
            STATS["export_failed"] += 1
            STATS["export_error"] = f"{name}: {e}"[:200]
            FAILED.append(name)
    gpu = next((t.device.index for t in tensors.values() if t is not None and t.is_cuda), 0)
    kv.set(key(slot), json.dumps({"owner": owner, "pid": os.getpid(), "gpu": gpu, "gen": time.time_ns(),
                                  "tensors": descs}))
    if slot not in slots(kv):
        kv.append("vram/slots", slot + ",")
    STATS["exported"] = len(descs)
    return len(descs)


def publish_warm(kv, slot: str, spec: dict | None) -> None:
    """The warm-up a standby should run for ``slot`` (operator/standby.py warm_device); None:
    only the generic small one."""
    kv.set(f"vram/warm/{slot}", json.dumps({"spec": spec}))


def read_warm(kv, slot: str) -> tuple[bool, dict | None]:
    """(published, spec) of ``slot``'s warm-up."""
    raw = kv.get_str(f"vram/warm/{slot}")
    if raw is None:
        return False, None
    return True, json.loads(raw).get("spec")


def standby_warm_on(kv, gpu, pending: bool = False) -> bool | None:
    """None: no standby is parked (``standby/roster``, kept by the operator); True: one of the
    parked standbys has run its warm-up on ``gpu`` (an int, "cpu" or None); False: not yet.
    ``pending``: a standby the operator spawned that is still starting (``standby/pending``)
    counts as "not yet" -- for a job's first workers, which would otherwise race it; never for
    a replacement, whose first step must not wait for the refill standby spawned behind it."""
    names = roster(kv)
    if not names:
        return False if (pending and (kv.get_str("standby/pending") or "")) else None
    where = ["any"] + ([f"gpu{gpu}"] if isinstance(gpu, int) else ["cpu"])
    return any(kv.exists(f"standby/warm/{n}/{w}") for n in names for w in where)


# Warm-up windows for a standby that arrives while the workers train (a refill after a takeover):
# its warm-up of a GPU must not run beside that GPU's training steps.  The standby files a request
# (``standby/warm_req/<name>`` = {"id", "gpus"}); the job master turns it into a runtime plan
# (``warm_window``), which every rank applies at the same committed step; the ranks on those GPUs
# grant it (``standby/warm_grant/<name>/gpu<g>``) and pause until the standby's warm key appears.
def request_warm_window(kv, name: str, req_id: int, gpus) -> None:
    kv.set(f"standby/warm_req/{name}", json.dumps({"id": int(req_id), "gpus": sorted(int(g) for g in gpus)}))


def read_warm_request(kv, name: str) -> dict | None:
    raw = kv.get_str(f"standby/warm_req/{name}")
    return json.loads(raw) if raw else None


def roster(kv) -> list[str]:
    return [n for n in (kv.get_str("standby/roster") or "").split(",") if n]


def publish_act(kv, slot: str, act_bytes: int, micro_batch: int, fixed_bytes: int = 0) -> None:
    """HBM one training step of ``slot`` needs beyond its persistent state; ``fixed_bytes`` of it
    do not shrink with a smaller micro-batch (transposed-weight caches, library workspaces)."""
    kv.set(f"vram/act/{slot}", json.dumps({"act_bytes": int(act_bytes), "micro_batch": int(micro_batch),
                                           "fixed_bytes": int(fixed_bytes)}))


def read_act(kv, slot: str) -> tuple[int, int, int]:
    """(act bytes, micro-batch, fixed bytes) ``slot``'s worker published; zeros if none."""
    raw = kv.get_str(f"vram/act/{slot}")
    if raw is None:
        return 0, 0, 0
    d = json.loads(raw)
    return int(d.get("act_bytes", 0)), int(d.get("micro_batch", 0)), int(d.get("fixed_bytes", 0))


def trained(kv, slot: str) -> bool:
    """``slot``'s worker has committed its first step (it published its step's HBM need)."""
    return kv.exists(f"vram/act/{slot}")


def slots(kv) -> list[str]:
    return sorted({s for s in (kv.get_str("vram/slots") or "").split(",") if s})


def import_published(kv, slot: str, held: dict | None = None) -> dict | None:
    """Standby: (re-)import the tensors published for worker ``slot``.  Returns {"owner", "pid",
    "gpu", "tensors"}, or ``held`` unchanged when nothing new was published."""
    raw = kv.get_str(key(slot))
    if raw is None:
        return held
    d = json.loads(raw)
    if held is not None and (held.get("owner"), held.get("pid"), held.get("gen")) == (
            d.get("owner"), d.get("pid"), d.get("gen")):
        return held
    # a new export (new process, or the same one after rebuilding its buffers): the old
    # imports go first, so memory the exporter has freed is not kept alive here
    if held is not None:
        held.get("tensors", {}).clear()
    if d.get("pid") is None or reaped(d["pid"]):
        return held     # never map the handles of a process that is gone (its memory may be freed)
    from easydl_amd.ps.ipc import import_tensor
    with torch.cuda.device(int(d.get("gpu", 0))):
        ts = {}
        for name, desc in d.get("tensors", {}).items():
            try:
                ts[name] = import_tensor(desc)
            except RuntimeError as e:
                log.warning("vram: cannot import %s from %s: %s", name, d.get("owner"), e)
    return {"owner": d.get("owner"), "pid": d.get("pid"), "gpu": int(d.get("gpu", 0)), "gen": d.get("gen"),
            "tensors": ts}


def dead(pid) -> bool:
    """True once the exporting process runs no more GPU work: reaped, or its address space
    is released (utils/procfs.py) -- only then may another process write its buffers."""
    from easydl_amd.utils.procfs import mm_released
    try:
        os.kill(int(pid), 0)
    except ProcessLookupError:
        return True
    except (PermissionError, TypeError, ValueError):
        return False
    return mm_released(int(pid))


def reaped(pid) -> bool:
    """True once ``pid`` is gone altogether (its parent has collected it): its teardown -- GPU
    queues included -- is complete.  A zombie does not count: when a last address-space
    reference is dropped late, the address space (and the GPU queues it holds) is torn down
    after the task already reads as a zombie."""
    try:
        os.kill(int(pid), 0)
    except ProcessLookupError:
        return True
    except (PermissionError, TypeError, ValueError):
        return False
    return False


ADOPTED_FROM: dict = {}          # {"pid": ...} of the process whose buffers were adopted


def adopt(tensors: dict[str, torch.Tensor], pid=None) -> None:
    """Takeover: these imported tensors back the next FlatParams / optimizer built here."""
    _ADOPTED.clear()
    _ADOPTED.update(tensors)
    TAKEN.clear()
    ADOPTED_FROM.clear()
    if pid is not None:
        ADOPTED_FROM["pid"] = int(pid)


def take(name: str, numel: int, dtype: torch.dtype, device, keep: bool = False) -> torch.Tensor | None:
    """The adopted tensor for ``name`` if it matches (numel, dtype, device), else None.  Zero-filled,
    unless ``keep``: training state (weights, master, moments) keeps the dead worker's values, so a
    replacement can resume from them when its step marks say they are consistent
    (utils/stepmarks.py); otherwise a restore or state transfer overwrites them anyway."""
    t = _ADOPTED.pop(name, None)
    if t is None:
        return None
    dev = torch.device(device)
    if t.numel() != numel or t.dtype != dtype or t.device != dev:
        log.warning("vram: adopted %s does not match (%s %s %s vs %s %s %s): allocating", name, t.numel(), t.dtype,
                    t.device, numel, dtype, dev)
        return None
    if not keep:
        t.zero_()
    STATS["adopted"] += 1
    STATS["adopted_bytes"] += t.numel() * t.element_size()
    TAKEN[name] = t.data_ptr()
    return t


def adopted_dtype(prefix: str, suffix: str) -> torch.dtype | None:
    """dtype of an adopted tensor named ``prefix...suffix`` (``opt/``, ``/m``: the dead worker's
    Adam moment dtype, which its replacement must keep), None if there is none."""
    for name, t in _ADOPTED.items():
        if name.startswith(prefix) and name.endswith(suffix):
            return t.dtype
    return None


def pending(name: str) -> bool:
    """An adopted tensor of this name is waiting to be taken."""
    return name in _ADOPTED


def adopted_any() -> bool:
    """True if some buffer of this process was built on a dead worker's HBM."""
    return bool(TAKEN)


def missing(tensors) -> list[str]:
    """Names of ``(name, tensor)`` pairs whose storage is NOT an adopted buffer."""
    ptrs = set(TAKEN.values())
    return [n for n, t in tensors if t.data_ptr() not in ptrs]


def release_unused() -> list[str]:
    """Drop adopted tensors nothing took (their memory goes back to the driver); returns their
    names (a name or size mismatch, e.g. another gradient dtype, or an optimizer without
    that state)."""
    names = sorted(_ADOPTED)
    _ADOPTED.clear()
    return names
