"""Checkpointing: format v1, sharded asynchronous in-memory snapshots, disk persistence.

Capability: "resume the training" after failures (reference README.md:27) and
the north star's "in-memory async checkpoint to host DRAM via pinned
hipMemcpyAsync on a side stream" (BASELINE.json).

**Format v1** (``edl-ckpt/1``).  A checkpoint of step N is a directory
``step-<N>/`` with ``manifest.json`` and one ``shard-<r>-of-<W>.bin`` per shard.
The manifest lists every state tensor (flat parameter buffers, fp32 master,
moments) with dtype, total numel and, per shard, the element range [lo, hi)
and byte offset inside the shard file; plus scalars (step, optimizer step,
epoch, world, RNG seed) and a 64-bit checksum per shard.  The byte layout of a
shard file is *identical* to the shared-memory slot, so persisting is one
``write`` and restoring is ``mmap`` + H2D.

**Sharded in-memory snapshots.**  DDP state is replicated, so rank r of W
snapshots only its 1/W slice of every flat buffer (8B Llama: 112 GB of state
-> 14 GB per rank at 8 GPUs).  Slices go through the native engine
(csrc/runtime/shm_store.cpp): event on the compute stream after the optimizer,
low-priority side stream, chunked hipMemcpyAsync into the free A/B slot of a
page-locked ``/dev/shm`` segment, committer thread publishes the slot.  The
next optimizer step waits on the copy (``fence``), so the snapshot overlaps
forward+backward and is always a consistent post-step state.  Segments live
in ``/dev/shm`` and survive worker death (the operator unlinks them at job
end); restoring the full state needs all W shards of one step, which the A/B
slots make available even while a new snapshot is being written.
"""
from __future__ import annotations

import ctypes
import glob
import json
import logging
import os
import re
import threading
import time

import numpy as np
import torch
import torch.distributed as dist

from easydl_amd import _native

log = logging.getLogger(__name__)

FORMAT = "edl-ckpt/1"
ALIGN = 4096
_DT = {torch.bfloat16: "bfloat16", torch.float32: "float32", torch.float16: "float16", torch.int64: "int64"}
_TD = {v: k for k, v in _DT.items()}


def _align(n: int) -> int:
    return (n + ALIGN - 1) // ALIGN * ALIGN


# ---------------------------------------------------------------------------- checksum
def checksum_np(buf: np.ndarray, base_index: int = 0) -> int:
    """Reference of the GPU checksum: sum_i w_i*(2i+1) mod 2^64 over uint32 words."""
    w = np.frombuffer(buf.tobytes() if not buf.flags["C_CONTIGUOUS"] else buf, dtype=np.uint32).astype(np.uint64)
    idx = np.arange(base_index, base_index + w.size, dtype=np.uint64)
    with np.errstate(over="ignore"):
        return int(np.sum(w * (2 * idx + 1), dtype=np.uint64))


def checksum_tensor(t: torch.Tensor, out: torch.Tensor | None = None, base_index: int = 0) -> torch.Tensor:
    """Checksum of a contiguous tensor's bytes; on GPU returns a device int64 tensor (no sync)."""
    if t.is_cuda:
        k = _native.kernels()
        if out is None:
            out = torch.zeros(1, dtype=torch.int64, device=t.device)
        k.check("edl_checksum", t.data_ptr(), t.numel() * t.element_size(), out.data_ptr(), base_index,
                _native.stream_of(t))
        return out
    v = checksum_np(t.detach().contiguous().view(torch.uint8).numpy(), base_index)
    r = torch.tensor([v - (1 << 64) if v >= (1 << 63) else v], dtype=torch.int64)
    if out is not None:
        out.add_(r)
        return out
    return r


# ---------------------------------------------------------------------------- layout
def shard_layout(tensors: list[tuple[str, torch.Tensor]], rank: int, world: int) -> tuple[list[dict], int]:
    """Per tensor the element range owned by ``rank`` and its byte offset in the shard."""
    out, off = [], 0
    for name, t in tensors:
        n = t.numel()
        lo, hi = n * rank // world, n * (rank + 1) // world
        nbytes = (hi - lo) * t.element_size()
        out.append({"name": name, "dtype": _DT[t.dtype], "numel": n, "lo": lo, "hi": hi, "offset": off,
                    "nbytes": nbytes})
        off = _align(off + nbytes)
    return out, off  # off = checksum trailer offset


class ShmSegment:
    """Python handle of one /dev/shm A/B segment (csrc/runtime/shm_store.cpp)."""

    def __init__(self, name: str, slot_bytes: int = 0, create: bool = True, pin: bool = False, nslots: int = 2):
        self.rt = _native.runtime()
        self.name = name
        self.h = self.rt("edl_shm_open", name.encode(), slot_bytes, nslots, 1 if create else 0)
        if not self.h:
            raise OSError(f"cannot open shm segment {name}")
        self.slot_bytes = self.rt("edl_shm_slot_bytes", self.h)
        self.pinned = False
        if pin:
            rc = self.rt("edl_shm_pin", self.h)
            self.pinned = rc == 0
            if rc != 0:
                log.warning("hipHostRegister of %s failed (%d): D2H copies will be pageable", name, rc)

    def data(self, slot: int) -> int:
        return self.rt("edl_shm_data", self.h, slot)

    def view(self, slot: int, offset: int, nbytes: int) -> np.ndarray:
        addr = self.data(slot) + offset
        return np.ctypeslib.as_array((ctypes.c_uint8 * nbytes).from_address(addr))

    def slot_info(self, slot: int) -> dict | None:
        step, epoch, nb, cs = ctypes.c_int64(), ctypes.c_int64(), ctypes.c_uint64(), ctypes.c_uint64()
        meta = ctypes.create_string_buffer(4096)
        st = self.rt("edl_shm_slot_info", self.h, slot, ctypes.byref(step), ctypes.byref(epoch), ctypes.byref(nb),
                     ctypes.byref(cs), meta, 4096)
        if st != 2:
            return None
        return {"slot": slot, "step": step.value, "epoch": epoch.value, "nbytes": nb.value, "checksum": cs.value,
                "meta": json.loads(meta.value.decode() or "{}")}

    def committed(self) -> list[dict]:
        return [i for s in range(2) if (i := self.slot_info(s)) is not None]

    def begin(self) -> int:
        return self.rt("edl_shm_begin", self.h)

    def commit(self, slot, step, epoch, nbytes, checksum, meta: dict):
        rc = self.rt("edl_shm_commit", self.h, slot, step, epoch, nbytes, checksum & ((1 << 64) - 1),
                     json.dumps(meta, separators=(",", ":")).encode())
        if rc != 0:
            raise OSError(-rc, "shm commit failed (meta too large?)")

    def populate_async(self, threads: int = 16) -> bool:
        """Fault every slot's pages in on background threads (csrc: edl_shm_populate_async)."""
        return self.rt("edl_shm_populate_async", self.h, threads) == 0

    def populated(self, slot: int | None = None) -> bool:
        """False while a background population is still running (``slot``: only as far as the
        end of that slot; population runs slot 0 first, and a straggling piece of it is just
        faulted in by the copy)."""
        total = ctypes.c_uint64()
        done = self.rt("edl_shm_populate_progress", self.h, ctypes.byref(total))
        if slot is not None and total.value:
            return done >= min(total.value, (slot + 1) * self.slot_bytes)
        return done >= total.value

    def close(self, unlink: bool = False):
        if self.h:
            self.rt("edl_shm_close", self.h, 1 if unlink else 0)
            self.h = None


# Segments a hot standby mapped and pre-faulted before any failure
# (easydl_amd/operator/standby.py); a restore in the same process reuses them.
_PREMAPPED: dict[str, ShmSegment] = {}


def premap_job_segments(job: str, threads: int = 8) -> list[str]:
    """Map + pre-fault every snapshot segment of ``job`` not mapped yet (returns the new names)."""
    new = []
    pat = re.compile(rf"^edl-{re.escape(job)}(-t\d+of\d+)?-w\d+-s\d+$")
    for path in sorted(glob.glob(f"/dev/shm/edl-{job}-*")):
        base = os.path.basename(path)
        name = "/" + base
        if not pat.match(base) or name in _PREMAPPED:
            continue
        try:
            seg = ShmSegment(name, create=False)
        except OSError:
            continue
        seg.rt("edl_shm_prefault", seg.h, threads)
        _PREMAPPED[name] = seg
        new.append(name)
    return new


def _open_segment(name: str) -> ShmSegment:
    seg = _PREMAPPED.pop(name, None)
    return seg if seg is not None else ShmSegment(name, create=False)


class CheckpointManager:
    """Periodic sharded in-memory snapshots (+ optional disk persistence) for a trainer.

    Args:
        job: job name (segment names ``/edl-<job>-w<W>-s<r>``).
        interval: snapshot every ``interval`` committed steps (Brain sets it so
            the D2H stays under ~5 % of step time).
        persist_dir: if set, every ``persist_every`` snapshots are also written
            to ``<persist_dir>/step-<N>/`` in format v1 (background thread).
        sharded: each rank stores 1/W of the replicated state (DDP).
        host_budget_gb: host DRAM one rank's two snapshot slots may take (default:
            ``EDL_CKPT_HOST_GB``, else ``host_fraction`` of min(MemAvailable, free
            /dev/shm) split over the node's ranks).
        lean: "auto" | "never" | "always" — a lean snapshot keeps the weights
            (fp32 master) and drops the optimizer moments (8 of AdamW's 12 B/param).

    Host-DRAM sizing: a DDP rank snapshots 1/W of the replicated
    state, but a tensor-parallel rank's shard is unique (Llama-3 70B at TP=8:
    ~105 GB per rank of master + moments, ~1.7 TB for the node's A/B slots).  At
    the first snapshot of each layout the DP group agrees (MAX over ranks) on the
    mode: ``full`` if every rank's two slots fit its budget, ``lean`` if the
    master-only slots fit, else ``off`` (no in-memory snapshots; disk persistence
    and survivor state transfer still work).  Restoring a lean snapshot zeroes the
    moments and restarts Adam's bias correction from that step
    (``FlatAdamW.moment_origin``) — a warm restart of the moments, not bit-exact.
    """

    def __init__(self, job: str, interval: int = 10, persist_dir: str | None = None, persist_every: int = 0,
                 sharded: bool = True, pin: bool | None = None, host_budget_gb: float | None = None,
                 host_fraction: float = 0.8, lean: str = "auto"):
        self.job = job
        env = os.environ.get("EDL_CKPT_HOST_GB")
        self.host_budget_gb = host_budget_gb if host_budget_gb is not None else (float(env) if env else None)
        self.host_fraction = host_fraction
        self.lean = os.environ.get("EDL_CKPT_LEAN", lean)
        self.mode = None            # "full" | "lean" | "off", agreed per layout (see _decide_mode)
        self._mode_key = None
        self.interval = max(1, interval)
        self.persist_dir = persist_dir
        self.persist_every = persist_every
        self.sharded = sharded
        # Page-locked slots (EDL_SNAPSHOT_PIN=1): snapshots DMA straight into the shm pages,
        # at the price of hipHostRegister on the first snapshot of a process (seconds for a
        # ~100 GB slot pair, serialised with the training thread's HIP calls) and of the
        # unpinning when the process dies.  0: slots stay pageable; snapshots stream through
        # a small pinned staging ring (csrc/runtime/shm_store.cpp run_staged).  A segment a
        # restore adopted is never pinned (see restore_latest).
        self.pin = pin if pin is not None else os.environ.get("EDL_SNAPSHOT_PIN", "0") == "1"
        # Pageable slots are populated on background threads as soon as the segment exists
        # (EDL_SHM_POPULATE_THREADS, 0 = never); the first snapshot waits for what is left.  A
        # segment adopted by a restore skips snapshots until its population is done instead:
        # the restored slot already holds a valid snapshot, and recovery should not stall.
        self.populate_threads = int(os.environ.get("EDL_SHM_POPULATE_THREADS", 4))
        self._skip_populating = False
        self._verify = None         # pending post-teardown check of an early hand-over (fence)
        self._deferred: list = []   # moment copies of the last restore still running (complete_restore)
        self._deferred_segs: list = []
        self._marks_check = None    # background post-reap check of an HBM resume
        self._seg: ShmSegment | None = None
        self._seg_key = None
        self._old_name = None       # previous layout's name of a relinked segment (see _segment)
        self._engine = None
        self._engine_dev = None
        self._ticket = None
        self._n = 0
        self._persist_thread = None
        self._persist_slot = None   # slot the persist thread is reading (None: idle)
        self._last_slot = None      # slot of the newest snapshot
        self.last_snapshot_step = None
        self.stats = {"snapshots": 0, "d2h_bytes": 0}

    # -- naming --------------------------------------------------------------
    # ``tag`` separates independent state sets of one job: with tensor
    # parallelism every TP rank's parameter shard is its own set ("-t<i>of<T>"),
    # each replicated over (and sharded across) that rank's DP group.
    def seg_name(self, world: int, shard: int, tag: str = "") -> str:
        return f"/edl-{self.job}{tag}-w{world}-s{shard}"

    @staticmethod
    def _tag(trainer) -> str:
        return getattr(trainer, "ckpt_tag", "") or ""

    @staticmethod
    def _comm(trainer):
        """The communicator the state is replicated over (DP group under TP)."""
        return getattr(trainer, "dp_comm", None) or trainer.comm

    @staticmethod
    def state_of(trainer) -> list[tuple[str, torch.Tensor]]:
        """Tensors that fully determine training state.  Where the optimizer keeps
        an fp32 master copy, the bf16 model buffer is NOT stored (it is
        bf16(master) by construction) — 14 % less snapshot traffic."""
        opt = trainer.opt.state_tensors()
        out = [(f"model.{g.name}", g.data) for g in trainer.flat.groups if f"opt.{g.name}.master" not in opt]
        out += list(opt.items())
        bufs = getattr(trainer, "bufs", None)
        if bufs is not None:
            out += [(f"model.buffers.{k}", t) for k, t in bufs.tensors.items()]
        return out

    @staticmethod
    def _moment_names(trainer) -> set:
        fn = getattr(trainer.opt, "moment_names", None)
        return set(fn()) if fn is not None else set()

    @staticmethod
    def _restore_scalars(trainer, meta: dict) -> None:
        """Step counters of a restored snapshot; a lean one restarts the moments."""
        trainer.step = int(meta["step"])
        trainer.opt.step_count = int(meta["opt_step"])
        if meta.get("lean"):
            st = trainer.opt.state_tensors()
            with torch.no_grad():
                for n in CheckpointManager._moment_names(trainer):
                    st[n].zero_()
            origin = trainer.opt.step_count
        else:
            origin = int(meta.get("moment_origin", 0))
        if hasattr(trainer.opt, "moment_origin"):
            trainer.opt.moment_origin = origin

    def resume_from_hbm(self, trainer, step: int, verify: dict | None = None) -> str:
        """The weights / master / moments in HBM are exactly the state after ``step`` (adopted
        from a dead worker whose step marks say no update was in flight, utils/stepmarks.py).
        Only the host-side counters and host state are set: from the newest snapshot at or
        before ``step`` (seed, LR schedule, moment origin), advanced to ``step``."""
        found = self.find_latest(self._tag(trainer), max_step=step)
        trainer.step = int(step)
        self._skip_populating = True    # recovering: a snapshot skips rather than waits for pages
        if verify is not None:
            # re-read the marks once the dead worker is gone, without holding up training; no
            # snapshot is taken meanwhile, and a failed check stops this process at the next
            # optimizer step (its replacement then restores from /dev/shm)
            self._marks_check = {"result": None}
            threading.Thread(target=self._check_marks_after_reap, args=(verify, self._marks_check),
                             name="edl-marks-check", daemon=True).start()
        if found is None:
            trainer.opt.step_count = int(step)
            return f"hbm:step{step}"
        meta = found[2][0]["meta"]
        trainer.opt.step_count = int(meta["opt_step"]) + (int(step) - int(meta["step"]))
        if hasattr(trainer.opt, "moment_origin"):
            trainer.opt.moment_origin = int(meta.get("moment_origin", 0))
        _load_host_state(trainer, meta.get("host"))
        return f"hbm:step{step}"

    @staticmethod
    def finish_restore(trainer) -> None:
        opt = trainer.opt.state_tensors()
        with torch.no_grad():
            for g in trainer.flat.groups:
                mk = f"opt.{g.name}.master"
                if mk in opt:
                    g.data.copy_(opt[mk])

    def _segment(self, world, shard, need_bytes, pin=True, tag: str = "", alloc_bytes: int = 0) -> ShmSegment:
        """The shm segment for this (world, shard, tag) layout.

        Page-locking a multi-GB slot (hipHostRegister) takes seconds and serialises
        with the training thread's HIP calls, so after a world change the mapped,
        pinned segment is re-used whenever it is big enough: its slots are
        invalidated and the file renamed to the new layout's name
        (edl_shm_reassign).  The first segment is sized for ``alloc_bytes`` (>= the
        shard of a world one rank smaller), so a shrink by one rank never re-pins."""
        key = (world, shard, tag)
        if self._seg is not None and self._seg_key == key and self._seg.slot_bytes >= need_bytes:
            return self._seg
        name = self.seg_name(world, shard, tag)
        if self._seg is not None:
            # nothing may still read or write the mapping while it changes hands:
            # the in-flight D2H / committer (wait) and a disk persist (join)
            self.wait()
            self._join_persist()
            if self._seg.slot_bytes >= need_bytes:
                old = self._seg.name
                self._drop_old_name()
                rc = self._seg.rt("edl_shm_relink", self._seg.h, name.encode())
                if rc == 0:
                    # the old layout's newest snapshot stays readable under the old name
                    # until this rank's first new-layout snapshot has committed
                    self._old_name = old if old != name else None
                    self._seg.name, self._seg_key = name, key
                    self.stats["reassigned"] = self.stats.get("reassigned", 0) + 1
                    return self._seg
                log.warning("re-using snapshot segment as %s failed (%d): new segment", name, rc)
            self._seg.close()
            self._seg = None
        self._drop_old_name()
        self._seg = ShmSegment(name, max(need_bytes, alloc_bytes), create=True, pin=self.pin and pin)
        self._seg_key = key
        if not self._seg.pinned and self.populate_threads > 0:
            self._seg.populate_async(self.populate_threads)
        return self._seg

    @staticmethod
    def _kept_slot_next(seg) -> bool:
        """True once a new-layout snapshot is current: the next write targets the other
        (kept, old-layout) slot."""
        cur = seg.rt("edl_shm_current", seg.h)
        info = seg.slot_info(cur) if cur >= 0 else None
        return info is not None and info["meta"].get("world") is not None and \
            seg.name.endswith(f"-w{info['meta']['world']}-s{info['meta'].get('shard')}")

    def _drop_old_name(self) -> None:
        """Unlink the previous layout's name of a relinked segment (its kept slot is about
        to be overwritten, or the segment changes hands again)."""
        old = getattr(self, "_old_name", None)
        self._old_name = None
        if old:
            try:
                # only if the name still refers to THIS segment: after a shard permutation
                # another rank's relink may have taken the name for its own live segment
                fd = self._seg.rt("edl_shm_fd", self._seg.h) if self._seg is not None else -1
                mine = os.fstat(fd) if fd >= 0 else None
                st = os.stat("/dev/shm" + old)
                if mine is not None and (st.st_ino, st.st_dev) != (mine.st_ino, mine.st_dev):
                    log.info("snapshot name %s now belongs to another segment: kept", old)
                    return
                os.unlink("/dev/shm" + old)
            except OSError:
                pass

    # -- host-DRAM sizing ----------------------------------------------------------
    def host_budget_bytes(self, trainer) -> int:
        """Host bytes this rank's snapshot slots may occupy."""
        if self.host_budget_gb is not None:
            return int(self.host_budget_gb * 2**30)
        avail = _meminfo_bytes("MemAvailable")
        try:
            st = os.statvfs("/dev/shm")
            avail = min(avail, st.f_bavail * st.f_frsize)
        except OSError:
            pass
        own = 2 * self._seg.slot_bytes if self._seg is not None else 0   # already counted as used
        ranks = int(os.environ.get("LOCAL_WORLD_SIZE") or 0) or int(getattr(trainer.comm, "world_size", 1) or 1)
        return int((avail + own) * self.host_fraction / max(1, ranks))

    def _decide_mode(self, trainer, comm, key, full_bytes: int, lean_bytes: int) -> str:
        """Agree (MAX over the group) on full / lean / off for this layout."""
        if self._mode_key == key and self.mode is not None:
            return self.mode
        budget = self.host_budget_bytes(trainer)
        if self.lean == "always":
            want = 1 if 2 * lean_bytes <= budget else 2
        elif 2 * full_bytes <= budget:
            want = 0
        elif self.lean != "never" and 2 * lean_bytes <= budget:
            want = 1
        else:
            want = 2
        agree = getattr(comm, "ctrl_all_reduce", None)
        # unsharded snapshots are rank 0's alone: nothing to agree with the others
        group = self.sharded and comm.world_size > 1 and agree is not None
        agreed = int(agree([float(want)], _MAX)[0]) if group else want
        self.mode = ("full", "lean", "off")[agreed]
        self._mode_key = key
        self.stats["mode"] = self.mode
        self.stats["host_budget_gb"] = round(budget / 2**30, 2)
        if self.mode != "full":
            log.warning("in-memory snapshots %s: two slots need %.1f GB (lean %.1f GB), budget %.1f GB per rank",
                        self.mode, 2 * full_bytes / 2**30, 2 * lean_bytes / 2**30, budget / 2**30)
        return self.mode

    # -- snapshot ------------------------------------------------------------
    def on_step(self, trainer) -> None:
        if trainer.step % self.interval:
            return
        if self.hbm_unverified():
            # resumed from a dead worker's HBM that is not verified yet: never let a snapshot
            # publish that state before the check
            self.stats["skipped_unverified"] = self.stats.get("skipped_unverified", 0) + 1
            return
        try:
            self.snapshot(trainer)
        except Exception as e:  # noqa: BLE001
            # a peer died inside the (first-of-layout) mode agreement: no snapshot this
            # step; the broken epoch is handed to the trainer's reconfiguration path
            comm = self._comm(trainer)
            from easydl_amd.parallel.comm import CommAborted
            if not isinstance(e, (CommAborted, RuntimeError)) or not (
                    getattr(comm, "aborted", False) or isinstance(e, CommAborted) or _comm_error(e)):
                raise
            log.warning("snapshot of step %d skipped: %s", trainer.step, e)
            self.stats["skipped_comm"] = self.stats.get("skipped_comm", 0) + 1
            if hasattr(comm, "abort"):
                comm.abort()

    def _plan(self, trainer):
        comm = self._comm(trainer)
        tag = self._tag(trainer)
        world = comm.world_size if self.sharded else 1
        shard = comm.rank if self.sharded else 0
        state = self.state_of(trainer)
        layout, cs_off = shard_layout(state, shard, world)
        moments = self._moment_names(trainer)
        lean_state = [(n, t) for n, t in state if n not in moments]
        headroom = lambda st: (max(shard_layout(st, s, world - 1)[1] for s in range(world - 1)) + 8  # noqa: E731
                               if world > 1 else 0)
        key = (world, shard, tag)
        sizes = (max(cs_off + 8, headroom(state)),
                 max(shard_layout(lean_state, shard, world)[1] + 8, headroom(lean_state)))
        return comm, tag, world, shard, state, layout, cs_off, lean_state, headroom, key, sizes

    def _own_key(self, trainer):
        """(world, shard, tag) of the segment this rank's snapshots go to (None: it writes none)."""
        comm = self._comm(trainer)
        if not self.sharded and comm.rank != 0:
            return None
        return ((comm.world_size, comm.rank) if self.sharded else (1, 0)) + (self._tag(trainer),)

    def prepare_layout(self, trainer) -> str | None:
        """Agree on this layout's full / lean / off mode now (the trainer calls it while
        entering an epoch, inside its failure handling), so no snapshot runs a collective;
        and create the layout's segment, so its pages are populated before the first
        snapshot needs them."""
        comm, tag, world, shard, state, _, _, lean_state, headroom, key, sizes = self._plan(trainer)
        if not self.sharded and comm.rank != 0:
            return None
        mode = self._decide_mode(trainer, comm, key, *sizes)
        if mode != "off" and state and state[0][1].is_cuda and self._ticket is None:
            # (with a snapshot still in flight, changing segments would first wait for its copy
            # -- 0.4 s of a 4-rank shrink's recovery in batch 30; the next snapshot does it)
            self._layout_segment(world, shard, tag, state if mode == "full" else lean_state, headroom)
        return mode

    def _layout_segment(self, world, shard, tag, state, headroom) -> ShmSegment:
        _, cs_off = shard_layout(state, shard, world)
        alloc = headroom(state) if world > 1 and self._seg is None else 0
        return self._segment(world, shard, cs_off + 8, pin=state[0][1].is_cuda, tag=tag, alloc_bytes=alloc)

    def snapshot(self, trainer) -> None:
        if self._deferred:
            self.complete_restore()   # the moments of the last restore are read below
        comm, tag, world, shard, state, layout, cs_off, lean_state, headroom, key, sizes = self._plan(trainer)
        if not self.sharded and comm.rank != 0:
            return
        mode = self._decide_mode(trainer, comm, key, *sizes)
        if mode == "off":
            self.stats["skipped_host"] = self.stats.get("skipped_host", 0) + 1
            return
        if mode == "lean":
            state = lean_state
            layout, cs_off = shard_layout(state, shard, world)
        self.wait()  # at most one snapshot in flight (and never one across a segment change)
        # (the first segment gets headroom: the largest shard of a world one rank smaller)
        seg = self._layout_segment(world, shard, tag, state, headroom)
        if not seg.populated(self._next_slot(seg)):
            if self._skip_populating:
                self.stats["skipped_populating"] = self.stats.get("skipped_populating", 0) + 1
                return
            t0 = time.perf_counter()
            while not seg.populated(self._next_slot(seg)):
                time.sleep(0.01)
            self.stats["populate_wait_s"] = round(self.stats.get("populate_wait_s", 0) + time.perf_counter() - t0, 3)
        if getattr(self, "_old_name", None) and self._kept_slot_next(seg):
            self._drop_old_name()   # this write overwrites the old layout's kept snapshot
        if self._persist_busy_slot(seg):
            # A/B slots: the slot this snapshot would overwrite is still being written to
            # disk (persisting takes longer than two intervals) -> skip rather than tear it
            self.stats["skipped"] = self.stats.get("skipped", 0) + 1
            return
        meta = {"format": FORMAT, "step": trainer.step, "opt_step": trainer.opt.step_count, "world": world,
                "shard": shard, "epoch": comm.epoch, "tag": tag, "host": _host_state(trainer),
                "lean": mode == "lean", "moment_origin": int(getattr(trainer.opt, "moment_origin", 0)),
                "t": [[d["name"], d["dtype"], d["numel"], d["lo"], d["hi"], d["offset"]] for d in layout]}
        dev = state[0][1].device
        if dev.type == "cuda":
            if self._engine is None or self._engine_dev != dev.index:
                self._engine = self.__class__._make_engine(dev.index)
                self._engine_dev = dev.index
            csum = torch.zeros(1, dtype=torch.int64, device=dev)
            ptrs, sizes, offs = [], [], []
            base = 0
            for (name, t), d in zip(state, layout):
                if d["nbytes"] == 0:
                    continue
                piece = t.view(-1)[d["lo"]:d["hi"]]
                checksum_tensor(piece, csum, base_index=d["offset"] // 4)
                ptrs.append(piece.data_ptr())
                sizes.append(d["nbytes"])
                offs.append(d["offset"])
            ptrs.append(csum.data_ptr())
            sizes.append(8)
            offs.append(cs_off)
            n = len(ptrs)
            arr = lambda v: (ctypes.c_uint64 * n)(*v)  # noqa: E731
            rt = _native.runtime()
            # the engine claims the non-current slot (edl_shm_begin); the previous
            # snapshot has been waited for, so "current" cannot move before it does
            self._last_slot = self._next_slot(seg)
            t = rt("edl_ckpt_snapshot", self._engine, seg.h, n, arr(ptrs), arr(sizes), arr(offs),
                   ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream), trainer.step, comm.epoch, cs_off,
                   json.dumps(meta, separators=(",", ":")).encode())
            if t < 0:
                raise RuntimeError(f"snapshot enqueue failed: hipError {-t}")
            self._ticket = t
            self._keep_alive = csum
        else:
            slot = seg.begin()
            self._last_slot = slot
            total = 0
            for (name, t), d in zip(state, layout):
                if d["nbytes"] == 0:
                    continue
                src = t.detach().view(-1)[d["lo"]:d["hi"]].contiguous().view(torch.uint8).numpy()
                seg.view(slot, d["offset"], d["nbytes"])[:] = src
                total += checksum_np(src, d["offset"] // 4)
            seg.commit(slot, trainer.step, comm.epoch, cs_off, total & ((1 << 64) - 1), meta)
        self.stats["snapshots"] += 1
        self.stats["d2h_bytes"] += cs_off
        self.last_snapshot_step = trainer.step
        self._n += 1
        if self.persist_dir and self.persist_every and self._n % self.persist_every == 0:
            self._persist_async(trainer.step)

    @staticmethod
    def _make_engine(device: int):
        # snapshot copies run as blit kernels: confine them to EDL_CKPT_CUS CUs (default 8,
        # one per XCD) so they barely touch the training kernels (csrc/runtime/shm_store.cpp)
        cus = int(os.environ.get("EDL_CKPT_CUS", 8))
        rt = _native.runtime()
        e = rt("edl_ckpt_engine_create", device, 256 << 20, cus)
        if not e:
            raise RuntimeError("cannot create checkpoint engine")
        rt("edl_ckpt_engine_staging", e, int(os.environ.get("EDL_CKPT_STAGE_MB", 128)) << 20,
           int(os.environ.get("EDL_CKPT_STAGES", 4)), int(os.environ.get("EDL_CKPT_COPY_THREADS", 16)))
        return e

    def _verify_handover(self) -> None:
        """After an early hand-over (operator/reconciler.py _early_replace) the restore wrote
        HBM adopted from a process the kernel had not finished tearing down.  Its GPU queues
        were gone (its address space was released first), but wait for the reap and check
        that the restored state is still exactly what the snapshot held, before the first
        optimizer step changes it: the master weights / moments by their checksum, the bf16
        weights against the master."""
        v, self._verify = self._verify, None
        from easydl_amd.utils import vram
        t0 = time.perf_counter()
        while not vram.reaped(v["pid"]) and time.perf_counter() - t0 < 120:
            time.sleep(0.005)
        for items, expect in v["shards"]:
            acc = torch.zeros(1, dtype=torch.int64, device=items[0][0].device)
            for dst, off in items:
                checksum_tensor(dst, acc, base_index=off // 4)
            got = int(acc.item()) & ((1 << 64) - 1)
            if got != expect:
                raise RuntimeError(f"restored state changed during the previous worker's teardown: {got:#x} != "
                                   f"{expect:#x}")
        tr = v["trainer"]
        for g, st in zip(tr.flat.groups, getattr(tr.opt, "state", [])):
            m = st.get("master")
            if m is not None and m is not g.data and not torch.equal(g.data, m.to(g.data.dtype)):
                raise RuntimeError(f"restored weights of {g.name} changed during the previous worker's teardown")
        self.stats["handover_verified_s"] = round(time.perf_counter() - t0, 3)

    def _check_marks_after_reap(self, v: dict, out: dict) -> None:
        """HBM resume: once the dead worker is gone, its step marks must still read (K, K) --
        had its GPU run another update on the adopted buffers after this process resumed from
        them, 'begin' would have moved."""
        from easydl_amd.utils import vram
        from easydl_amd.utils.stepmarks import read_slot
        t0 = time.perf_counter()
        while not vram.reaped(v["pid"]) and time.perf_counter() - t0 < 120:
            time.sleep(0.01)
        now = read_slot(v["job"], v["slot"], shadow=True)
        out["s"] = round(time.perf_counter() - t0, 3)
        ok = now is not None and now[:2] == v["marks"] and (v.get("shadow") is None or now[3:7] == v["shadow"])
        out["result"] = "ok" if ok else f"marks moved: {v['marks']} {v.get('shadow')} -> {now}"

    def hbm_unverified(self) -> bool:
        c = self._marks_check
        return c is not None and c["result"] is None

    def complete_restore(self, check: bool = True) -> None:
        """Join the deferred moment copies of the last restore (restore_latest ``defer_moments``):
        the current stream waits for them and the snapshot's checksum is verified as a whole.
        A mismatch raises before any update reads the moments."""
        pending, self._deferred = self._deferred, []
        segs, self._deferred_segs = self._deferred_segs, []
        try:
            for h in pending:
                t0 = time.perf_counter()
                h["thread"].join()
                if h["error"] is not None:
                    if check:
                        raise RuntimeError(f"deferred restore of {h['what']} failed: {h['error']}")
                    continue
                torch.cuda.current_stream(h["acc"].device).wait_event(h["event"])
                if check:
                    got = (int(h["acc"].item()) + int(h["acc2"].item())) & ((1 << 64) - 1)
                    if got != h["expect"]:
                        raise RuntimeError(f"checksum mismatch in {h['what']} (deferred moments): "
                                           f"{got:#x} != {h['expect']:#x}")
                self.stats["deferred_restore_wait_s"] = round(time.perf_counter() - t0, 3)
        finally:
            for seg in segs:
                threading.Thread(target=seg.close, name="edl-shm-unmap", daemon=True).start()

    def fence(self) -> None:
        """Make the current stream wait for the in-flight snapshot (call before the optimizer)."""
        if self._deferred:
            self.complete_restore()
        c = self._marks_check
        if c is not None and c["result"] is not None:
            self._marks_check = None
            if c["result"] != "ok":
                raise RuntimeError(f"HBM resume invalidated after the previous worker's teardown ({c['result']});"
                                   f" exiting so the replacement restores from the snapshot")
            self.stats["handover_verified_s"] = c["s"]
        if self._verify is not None:
            self._verify_handover()
        if self._ticket is not None and self._engine is not None:
            _native.runtime()("edl_ckpt_fence", self._engine, self._ticket,
                              ctypes.c_void_p(torch.cuda.current_stream().cuda_stream))

    def wait(self, timeout_s: float = 600.0) -> None:
        """Block until the in-flight snapshot is committed (main thread only)."""
        if self._ticket is not None and self._engine is not None:
            st = _native.runtime()("edl_ckpt_wait", self._engine, self._ticket, int(timeout_s * 1000))
            if st < 0:
                raise RuntimeError(f"snapshot failed: {st}")
            self._ticket = None
            if self._seg is not None and not self._seg.pinned:
                out = (ctypes.c_double * 4)()
                _native.runtime()("edl_ckpt_engine_staged_stats", self._engine, out)
                if out[2] > 0:
                    self.stats["staged_last"] = {"d2h_wait_s": round(out[0], 3), "copy_s": round(out[1], 3),
                                                 "total_s": round(out[2], 3), "mb": round(out[3] / 2**20, 1)}

    @staticmethod
    def _next_slot(seg: ShmSegment) -> int:
        cur = seg.rt("edl_shm_current", seg.h)
        return max(0, (cur + 1) % seg.rt("edl_shm_nslots", seg.h))

    def _persist_busy_slot(self, seg: ShmSegment) -> bool:
        th = self._persist_thread
        return (th is not None and th.is_alive() and self._persist_slot is not None
                and self._persist_slot == self._next_slot(seg))

    def _join_persist(self, timeout_s: float | None = None) -> None:
        th = self._persist_thread
        if th is not None and th is not threading.current_thread():
            th.join(timeout_s)

    # -- restore -------------------------------------------------------------
    def find_latest(self, tag: str = "", max_step: int | None = None) -> tuple[int, int, list[dict]] | None:
        """Newest step (<= ``max_step``) for which every shard of some world size has a committed slot."""
        best = None
        worlds = {}
        pat = re.compile(rf"^edl-{re.escape(self.job + tag)}-w(\d+)-s(\d+)$")
        for path in glob.glob(f"/dev/shm/edl-{self.job}{tag}-w*-s*"):
            base = os.path.basename(path)
            mt = pat.match(base)
            if mt is None:
                continue
            w, s = int(mt.group(1)), int(mt.group(2))
            worlds.setdefault(w, {})[s] = "/" + base
        for w, shards in worlds.items():
            if len(shards) != w:
                continue
            per = []
            for s in range(w):
                seg = ShmSegment(shards[s], create=False)
                # a relinked segment is visible under two layouts' names: keep the slots
                # whose recorded layout is the one this name stands for
                per.append({i["step"]: i for i in seg.committed()
                            if i["meta"].get("world", w) == w and i["meta"].get("shard", s) == s})
                seg.close()
            common = set(per[0])
            for p in per[1:]:
                common &= set(p)
            if max_step is not None:
                common = {c for c in common if c <= max_step}
            if common:
                st = max(common)
                if best is None or st > best[1]:
                    best = (w, st, [p[st] for p in per])
        return best

    def latest_step(self, trainer) -> int:
        """Newest restorable in-memory step of this trainer's state set (-1: none)."""
        self.wait()  # this rank's own in-flight snapshot counts once it is committed
        found = self.find_latest(self._tag(trainer))
        return -1 if found is None else found[1]

    def restore_latest(self, trainer, max_step: int | None = None, defer_moments: bool = False) -> str | None:
        """Restore the newest snapshot.  ``defer_moments`` (a rank that will not send its state
        to others before its first update, e.g. world 1): the Adam moments -- 2/3 of a full
        fp32 snapshot -- are copied under the first training step instead of before it
        (EDL_RESTORE_DEFER=0 turns that off); ``complete_restore`` (called by fence) joins them
        and verifies the whole checksum before the update reads them."""
        # Drain this rank's in-flight snapshot first: its D2H reads the very buffers the
        # restore is about to overwrite, and its commit must not publish a slot that
        # mixes pre- and post-rollback bytes under a pre-restore checksum.
        t_start = time.perf_counter()
        LAST_RESTORE_STATS.clear()
        self.complete_restore(check=False)
        self.wait()
        tag = self._tag(trainer)
        found = self.find_latest(tag, max_step)
        if found is None:
            if self.persist_dir:
                return self.load_dir_latest(trainer)
            return None
        world, step, infos = found
        t0 = time.perf_counter()
        state = dict(self.state_of(trainer))
        dev = next(iter(state.values())).device
        phases = {"find_s": round(t0 - t_start, 3)}
        own = self._own_key(trainer)
        verify = []
        later = frozenset()
        if (defer_moments and dev.type == "cuda" and not infos[0]["meta"].get("lean")
                and os.environ.get("EDL_RESTORE_DEFER", "1") == "1"):
            later = frozenset(self._moment_names(trainer))
        for s, info in enumerate(infos):
            t1 = time.perf_counter()
            seg = _open_segment(self.seg_name(world, s, tag))
            phases["open_s"] = round(phases.get("open_s", 0) + time.perf_counter() - t1, 3)
            keep = False
            try:
                loaded = _load_shard(lambda off, nb: seg.view(info["slot"], off, nb), info["meta"]["t"], state, dev,
                                     info["checksum"], f"shm shard {s} of step {step}", seg=seg, slot=info["slot"],
                                     later=later, deferred=self._deferred)
                if loaded is not None:
                    verify.append(loaded)
                # The segment this rank will write next (same layout, e.g. the only worker restarted):
                # keep the mapping as this rank's snapshot segment.  Unmapping ~100 GB of populated
                # pages costs seconds and takes the address-space lock the first step's allocations
                # need (3.1 s measured); re-mapping and page-locking it for the next snapshot would
                # cost seconds more.  It stays pageable: snapshots stream through the staging ring.
                keep = self._seg is None and own == (world, s, tag)
            finally:
                if keep:
                    self._seg, self._seg_key = seg, own
                    self.stats["adopted"] = self.stats.get("adopted", 0) + 1
                    if self.populate_threads > 0 and dev.type == "cuda":
                        # pages the dead writer never touched (a slot it was still filling) are
                        # allocated off the recovery path; snapshots wait for that by skipping
                        seg.populate_async(self.populate_threads)
                        self._skip_populating = True
                elif later:
                    self._deferred_segs.append(seg)   # closed once the deferred copy is done
                else:
                    threading.Thread(target=seg.close, name="edl-shm-unmap", daemon=True).start()
        t2 = time.perf_counter()
        self.finish_restore(trainer)
        if dev.type == "cuda":
            torch.cuda.current_stream(dev).synchronize()
        phases["finish_s"] = round(time.perf_counter() - t2, 3)
        LAST_RESTORE_STATS.update(phases)
        from easydl_amd.utils import vram
        pid = vram.ADOPTED_FROM.get("pid")
        if verify and pid is not None and not vram.reaped(pid):
            # this state lives in HBM adopted from a worker that is still being torn down
            # (early hand-over): re-verify it once that process is gone, before the first update
            self._verify = {"pid": pid, "shards": verify, "trainer": trainer}
        meta = infos[0]["meta"]
        self._restore_scalars(trainer, meta)
        _load_host_state(trainer, meta.get("host"))
        return f"shm{tag}:w{world}:step{step}"

    # -- disk persistence (format v1) ----------------------------------------------
    def _persist_async(self, step: int) -> None:
        if self._persist_thread is not None and self._persist_thread.is_alive():
            return
        # The thread owns (seg, slot) until it ends: snapshot() skips rather than reuse
        # that slot (_persist_busy_slot) and _segment() joins it before unmapping.
        self._persist_slot = self._last_slot
        args = (step, self._seg, self._engine, self._ticket, self._persist_slot)
        self._persist_thread = threading.Thread(target=self._persist, args=args, daemon=True)
        self._persist_thread.start()

    PERSIST_CHUNK = 64 << 20

    def _persist(self, step: int, seg: ShmSegment, engine, ticket, slot: int) -> None:
        try:
            if ticket is not None and engine is not None:
                # wait on the captured ticket: self._ticket belongs to the training thread
                if _native.runtime()("edl_ckpt_wait", engine, ticket, 600000) < 0:
                    return
            self._persist_slot_to_disk(step, seg, slot)
        except Exception:  # noqa: BLE001 - a failed persist must never kill training
            log.exception("persisting step %d failed", step)
        finally:
            self._persist_slot = None

    def _persist_slot_to_disk(self, step: int, seg: ShmSegment, slot: int) -> None:
        info = seg.slot_info(slot)
        if info is None or info["step"] != step:
            return
        m = info["meta"]
        tag = m.get("tag", "")
        d = os.path.join(self.persist_dir, f"step-{step}")
        os.makedirs(d, exist_ok=True)
        fname = f"shard{tag}-{m['shard']}-of-{m['world']}.bin"
        tmp = os.path.join(d, fname + ".tmp")
        src = seg.view(slot, 0, info["nbytes"])
        with open(tmp, "wb") as f:  # streamed from the mapping: no full-size host copy
            for o in range(0, info["nbytes"], self.PERSIST_CHUNK):
                f.write(src[o:o + self.PERSIST_CHUNK])
        after = seg.slot_info(slot)
        if after is None or any(after[k] != info[k] for k in ("step", "checksum", "nbytes")):
            os.unlink(tmp)  # the slot was rewritten under us: never publish a torn file
            log.warning("slot %d changed while persisting step %d: discarded", slot, step)
            return
        os.replace(tmp, os.path.join(d, fname))
        shard_manifest = {"file": fname, "checksum": info["checksum"], "nbytes": info["nbytes"],
                          "tensors": m["t"], "shard": m["shard"]}
        with open(os.path.join(d, f"shard{tag}-{m['shard']}.json"), "w") as f:
            json.dump(shard_manifest, f)
        if m["shard"] == 0:
            with open(os.path.join(d, f"manifest{tag}.json"), "w") as f:
                json.dump({"format": FORMAT, "step": step, "opt_step": m["opt_step"], "world": m["world"],
                           "epoch": m["epoch"], "host": m.get("host"), "lean": bool(m.get("lean")),
                           "moment_origin": int(m.get("moment_origin", 0)), "time": time.time()}, f)

    def load_dir_latest(self, trainer) -> str | None:
        dirs = sorted(glob.glob(os.path.join(self.persist_dir or "", "step-*")),
                      key=lambda p: int(p.rsplit("-", 1)[1]))
        tag = self._tag(trainer)
        for d in reversed(dirs):
            mf = os.path.join(d, f"manifest{tag}.json")
            if not os.path.exists(mf):
                continue
            m = json.load(open(mf))
            shards = [os.path.join(d, f"shard{tag}-{s}.json") for s in range(m["world"])]
            if not all(os.path.exists(p) for p in shards):
                continue
            try:
                load_dir(d, trainer, tag)
            except (RuntimeError, OSError, ValueError, KeyError) as e:
                # torn / truncated shard: fall back to the next older complete directory
                # (a later full load overwrites whatever this attempt already copied)
                log.warning("checkpoint %s unusable (%s): trying an older one", d, e)
                continue
            return f"disk:{d}"
        return None

    def close(self, unlink: bool = False) -> None:
        self.complete_restore(check=False)
        self.wait()
        self._join_persist(60)
        if unlink:
            self._drop_old_name()
        if self._seg is not None:
            self._seg.close(unlink)
            self._seg = None
        if self._engine is not None:
            _native.runtime()("edl_ckpt_engine_destroy", self._engine)
            self._engine = None


def load_dir(d: str, trainer, tag: str = "") -> None:
    """Cold resume from a format-v1 directory (any world size -> any world size)."""
    m = json.load(open(os.path.join(d, f"manifest{tag}.json")))
    state = dict(CheckpointManager.state_of(trainer))
    dev = next(iter(state.values())).device
    for s in range(m["world"]):
        sm = json.load(open(os.path.join(d, f"shard{tag}-{s}.json")))
        raw = np.memmap(os.path.join(d, sm["file"]), dtype=np.uint8, mode="r")
        _load_shard(lambda off, nb: np.array(raw[off:off + nb]), sm["tensors"], state, dev, sm["checksum"],
                    sm["file"])
    CheckpointManager.finish_restore(trainer)
    CheckpointManager._restore_scalars(trainer, m)
    _load_host_state(trainer, m.get("host"))


_MAX = dist.ReduceOp.MAX


def _meminfo_bytes(key: str) -> int:
    try:
        with open("/proc/meminfo") as f:
            for line in f:
                if line.startswith(key + ":"):
                    return int(line.split()[1]) * 1024
    except OSError:
        pass
    return 0


def _host_state(trainer) -> dict | None:
    fn = getattr(trainer, "host_state", None)
    return fn() if fn is not None else None


def _load_host_state(trainer, h) -> None:
    fn = getattr(trainer, "load_host_state", None)
    if fn is not None:
        fn(h)


LAST_RESTORE_STATS: dict = {}   # where the newest shm -> HBM restore spent its time (copy vs DMA wait)


def _restore_items(seg, slot, items, dev, stream, stats: dict) -> None:
    """Native pipelined shm -> HBM copy of ``items`` ((dst view, segment offset), ...) on ``stream``."""
    n = len(items)
    if n == 0:
        return
    arr = lambda v: (ctypes.c_uint64 * n)(*v)  # noqa: E731
    ptrs = [d.data_ptr() for d, _ in items]
    sizes = [d.numel() * d.element_size() for d, _ in items]
    offs = [o for _, o in items]
    cs = ctypes.c_void_p(stream.cuda_stream)
    if os.environ.get("EDL_RESTORE_V1") == "1":   # A/B: per-chunk threads, 2 stages of 256 MiB
        rc = _native.runtime()("edl_ckpt_restore_pipelined", seg.h, slot, n, arr(ptrs), arr(sizes), arr(offs),
                               cs, 256 << 20, 16)
    else:
        st = (ctypes.c_double * 4)()
        rc = _native.runtime()("edl_ckpt_restore_pipelined2", seg.h, slot, n, arr(ptrs), arr(sizes), arr(offs),
                               cs, int(os.environ.get("EDL_RESTORE_CHUNK_MB", 128)) << 20,
                               int(os.environ.get("EDL_RESTORE_THREADS", 16)),
                               int(os.environ.get("EDL_RESTORE_STAGES", 4)), st)
        stats.update(copy_s=round(st[0], 3), dma_wait_s=round(st[1], 3), total_s=round(st[2], 3),
                     gb=round(st[3] / 2**30, 2), gbps=round(st[3] / 2**30 / max(st[2], 1e-9), 1))
    if rc != 0:
        raise RuntimeError(f"pipelined restore failed: hipError {rc}")


def _load_shard(read, table, state, dev, expect: int, what: str, seg=None, slot=None, later=frozenset(),
                deferred: list | None = None) -> None:
    """Copy one shard's tensor slices to their device buffers and verify the checksum
    (on the GPU for device tensors: no host pass over tens of GB).  From a shm
    segment to a GPU the copy runs through the native pipelined restore
    (multi-threaded memcpy into pinned staging buffers overlapped with DMA).

    ``later`` (names; shm -> GPU only): those tensors -- the Adam moments, which nothing reads
    before the first optimizer update -- are copied by a background thread on a side stream
    while training resumes; their checksum half is folded in at ``deferred`` completion
    (CheckpointManager.complete_restore, before that update)."""
    for name, dt, numel, lo, hi, off in table:
        t = state.get(name)
        if t is None:
            raise RuntimeError(f"{what}: snapshot holds {name}, which this process's state does not have")
        if _DT[t.dtype] != dt or t.numel() != numel:
            # the bytes are copied raw: another dtype (e.g. bf16 vs fp32 Adam moments) or size
            # would load garbage under a matching checksum
            raise RuntimeError(f"{what}: {name} is {dt}[{numel}] in the snapshot but {_DT[t.dtype]}[{t.numel()}] "
                               "here (moment dtype / model mismatch); refusing to restore")
    acc = torch.zeros(1, dtype=torch.int64, device=dev) if dev.type == "cuda" else None
    if acc is not None and seg is not None:
        now, items_later = [], []
        for name, dt, numel, lo, hi, off in table:
            t = state[name]
            if (hi - lo) * t.element_size():
                (items_later if name in later and deferred is not None else now).append((t.view(-1)[lo:hi], off))
        _restore_items(seg, slot, now, dev, torch.cuda.current_stream(dev), LAST_RESTORE_STATS)
        t_cs = time.perf_counter()
        for dst, off in now:
            checksum_tensor(dst, acc, base_index=off // 4)
        if items_later:
            from easydl_amd.utils.resources import new_stream
            side = new_stream(dev)
            acc2 = torch.zeros(1, dtype=torch.int64, device=dev)
            ev = torch.cuda.Event()
            nb = sum(d.numel() * d.element_size() for d, _ in items_later)
            h = {"acc": acc, "acc2": acc2, "event": ev, "expect": expect, "what": what, "error": None,
                 "bytes": nb, "stats": {}}

            def run():
                try:
                    with torch.cuda.device(dev), torch.cuda.stream(side):
                        _restore_items(seg, slot, items_later, dev, side, h["stats"])
                        for dst, off in items_later:
                            checksum_tensor(dst, acc2, base_index=off // 4)
                        ev.record(side)
                except Exception as e:  # noqa: BLE001 - reported at completion, before the update
                    h["error"] = e

            h["thread"] = threading.Thread(target=run, name="edl-restore-deferred", daemon=True)
            h["thread"].start()
            deferred.append(h)
            LAST_RESTORE_STATS["deferred_bytes"] = LAST_RESTORE_STATS.get("deferred_bytes", 0) + nb
            return now + items_later, expect
        got = int(acc.item()) & ((1 << 64) - 1)
        LAST_RESTORE_STATS["checksum_s"] = round(time.perf_counter() - t_cs, 3)
        if got != expect:
            raise RuntimeError(f"checksum mismatch in {what}: {got:#x} != {expect:#x}")
        return now, expect
    total = 0
    for name, dt, numel, lo, hi, off in table:
        t = state[name]
        nbytes = (hi - lo) * t.element_size()
        if nbytes == 0:
            continue
        host = read(off, nbytes)
        dst = t.view(-1)[lo:hi]
        dst.copy_(torch.from_numpy(host).view(_TD[dt]))
        if acc is not None:
            checksum_tensor(dst, acc, base_index=off // 4)
        else:
            total += checksum_np(host, off // 4)
    got = (int(acc.item()) if acc is not None else total) & ((1 << 64) - 1)
    if got != expect:
        raise RuntimeError(f"checksum mismatch in {what}: {got:#x} != {expect:#x}")


def unlink_job_segments(job: str) -> int:
    n = 0
    pat = re.compile(rf"^edl-{re.escape(job)}((-t\d+of\d+)?-w\d+-s\d+|-(marks|gshadow)-[a-z]+\d+|-ps\d+)$")
    for path in glob.glob(f"/dev/shm/edl-{job}-*"):
        if not pat.match(os.path.basename(path)):
            continue
        try:
            os.unlink(path)
            n += 1
        except OSError:
            pass
    return n


def _comm_error(e: Exception) -> bool:
    from easydl_amd.parallel.errors import is_comm_error
    return is_comm_error(e)
