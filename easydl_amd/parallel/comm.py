"""Epoch-scoped communicators.

A :class:`Communicator` is one rank's membership in ONE rendezvous epoch.  It
owns a data-plane process group (RCCL — ``ProcessGroupNCCL`` is RCCL on ROCm —
for GPU tensors, gloo for CPU tensors) and a gloo control-plane group for
small CPU agreements (step agreement, votes).  Groups are constructed directly
on a ``PrefixStore("edl/<job>/e<epoch>")`` of the job's TCPStore, so a new
epoch never collides with the old one and no global ``init_process_group``
state has to be torn down: on a membership change the old communicator is
``abort()``-ed (unblocking any rank stuck in a collective with a dead peer)
and a fresh one is built for the new world.

xGMI note: a node's 8 MI355X GPUs are fully connected point-to-point (7 links
per GPU); RCCL's multi-channel rings/trees already spread traffic over the
links, and large buckets (>=64 MiB, Brain-tunable) keep every link busy.
"""
from __future__ import annotations

import datetime
import logging
import math
import os
import threading
import time

import torch
import torch.distributed as dist

log = logging.getLogger(__name__)


class CommAborted(RuntimeError):
    """A collective was aborted because membership changed or a peer died."""


class CollectiveMismatch(RuntimeError):
    """Ranks issued different collectives at the same position (EDL_CHECK_COLLECTIVES=1)."""


def _signature(kind: str, t: torch.Tensor, extra: int = 0) -> int:
    """31-bit fingerprint of (kind, numel, dtype, extra) — identical on every rank for the same call."""
    import zlib
    return zlib.crc32(f"{kind}:{t.numel()}:{t.dtype}:{extra}".encode()) & 0x7FFFFFFF


def _ranks_per_device(store, rank: int, world: int, device) -> int:
    """The most ranks any one GPU carries in this group (device UUIDs through the store)."""
    uuid = str(torch.cuda.get_device_properties(device).uuid)
    store.set(str(rank), uuid)
    seen: dict[str, int] = {}
    for p in range(world):
        u = uuid if p == rank else store.get(str(p)).decode()
        seen[u] = seen.get(u, 0) + 1
    return max(seen.values())


def _td(s: float) -> datetime.timedelta:
    return datetime.timedelta(seconds=s)


def _rccl_nonblocking(opts, reformed: bool) -> bool:
    """Non-blocking RCCL communicator init where this torch exposes the config field.
    ``EDL_RCCL_NONBLOCKING``: "auto" (default) for epochs re-formed after a failure or a
    membership change only -- the recovery path, where an abort must be able to end an init in
    progress -- while a job's first epoch keeps RCCL's default blocking init; "1" always; "0"
    never."""
    mode = os.environ.get("EDL_RCCL_NONBLOCKING", "auto")
    if mode == "0" or (mode != "1" and not reformed):
        return False
    cfg = getattr(opts, "config", None)
    if cfg is None or not hasattr(cfg, "blocking"):
        return False
    cfg.blocking = 0
    return True


class Communicator:
    def __init__(self, store: dist.Store, rank: int, world_size: int, epoch: int, *, device: torch.device,
                 job: str = "job", timeout_s: float = 120.0, control_timeout_s: float = 30.0,
                 high_priority: bool = True, tag: str = "", data: bool = True, data_backend: str | None = None,
                 xgmi_factory=None, probe: str = "now"):
        self.rank = rank
        self.world_size = world_size
        self.epoch = epoch
        self.device = torch.device(device)
        self.tag = tag
        self.xgmi = None
        self.xgmi_mode = None
        self.xgmi_probe: dict | None = None
        self.allreduce_policy: dict | None = None
        # "auto" all-reduce policy source (see warmup()): "now" probes inside warmup() unless a
        # policy for this (group, world) is cached; "defer" (re-formations: the recovery
        # critical path) never probes there -- RCCL only until run_deferred_probe() after the
        # epoch's first committed step, or a cached / Brain policy adopted at once
        self.probe_mode = probe
        self.probe_pending = False
        self.group = "".join(ch for ch in tag if not ch.isdigit()) or "dp"
        self._root_store, self._job = store, job
        self._aborted = False
        self._lock = threading.Lock()
        # debug: verify every rank issues the same collective sequence (the classic
        # DDP hang: one rank's bucket order or sizes differ) — SURVEY.md §5.2
        self.check = os.environ.get("EDL_CHECK_COLLECTIVES", "0") == "1"
        self._seq = 0
        t0 = time.perf_counter()
        base = dist.PrefixStore(f"edl/{job}/e{epoch}" + (f"/{tag}" if tag else ""), store)
        self.ctrl = dist.ProcessGroupGloo(dist.PrefixStore("ctrl", base), rank, world_size, _td(control_timeout_s))
        # default "auto": at world > 1 the hand-written xGMI engine is measured against
        # RCCL at the start of every epoch and kept for the message sizes where it wins
        data_backend = data_backend or os.environ.get("EDL_COMM", "auto")
        self.xgmi_min_bytes = 0         # all-reduces (in place, registered) at least this large -> engine
        self.xgmi_min_bytes_staged = 0  # ... and through the staging workspace
        # "auto-gloo" (tests): the auto engine/probe path with gloo on GPU tensors standing in
        # for RCCL, so several ranks can share one GPU (RCCL refuses duplicate devices)
        self.data_kind = "rccl"
        self.nonblocking = False
        if data_backend == "auto-gloo":
            data_backend, self.data_kind = "auto", "gloo"
        if not data:
            self.data = None
            self.backend = self.data_kind = "none"
        elif self.device.type == "cuda" and data_backend == "xgmi-only":
            # the hand-written engine is the ONLY data plane (no RCCL communicator): several
            # ranks may then share one GPU (RCCL refuses duplicate devices), e.g. to exercise
            # worker death + shrink on a single MI355X.  broadcast = all-reduce of a buffer
            # that only the source holds; unsupported dtypes go through the CPU control plane.
            from easydl_amd.parallel.xgmi import XgmiComm
            self.data = None
            self.xgmi = XgmiComm(dist.PrefixStore("xgmi", base), "ws", rank, world_size, self.device,
                                 timeout_s=timeout_s)
            self.xgmi_mode = "xgmi"
            self.backend = self.data_kind = "xgmi"
        elif self.device.type == "cuda":
            if (data_backend == "auto" and world_size > 1 and os.environ.get("EDL_XGMI_CROSS_GPU", "0") != "1"
                    and _ranks_per_device(dist.PrefixStore("devs", base), rank, world_size, self.device) == 1):
                # every rank on its own GPU: the engine's peer reads over xGMI between GPUs have
                # not run on hardware yet (only ranks sharing one GPU have), so "auto" keeps RCCL
                # there; EDL_XGMI_CROSS_GPU=1 (or EDL_COMM=xgmi) lets the probe decide
                self.xgmi_probe = {"selected": "rccl", "reason": "one rank per GPU; EDL_XGMI_CROSS_GPU=1 probes"}
                data_backend = "rccl"
            if data_backend in ("xgmi", "auto") and world_size > 1:
                # csrc/kernels/xgmi.hip: abortable direct all-reduce over IPC-mapped peer
                # memory; RCCL keeps the other collectives (and all-reduce in "auto" until
                # warmup() has measured both on this node and per message size)
                if xgmi_factory is None:
                    from easydl_amd.parallel.xgmi import XgmiComm as xgmi_factory
                try:
                    # the engine's bounded waits: a peer that never arrives (or a mapping that does not
                    # work between two GPUs) ends a collective after this long, not after the data
                    # plane's full timeout -- the probe then keeps RCCL
                    eng_timeout = min(timeout_s, float(os.environ.get("EDL_XGMI_TIMEOUT_S", 30)))
                    self.xgmi = xgmi_factory(dist.PrefixStore("xgmi", base), "ws", rank, world_size, self.device,
                                             timeout_s=eng_timeout)
                    self.xgmi_mode = data_backend
                except Exception as e:  # noqa: BLE001
                    if data_backend == "xgmi":
                        raise
                    # auto: the engine is an optimisation; RCCL alone is always correct
                    log.warning("xGMI engine unavailable (%s); RCCL only", e)
                    self.xgmi_probe = {"selected": "rccl", "error": str(e)[:200]}
                    self.xgmi = None
                if data_backend == "auto":
                    # the engine is used by every rank or by none: a rank whose mapping failed
                    # (hipIpcOpenMemHandle, after every handle was published) falls back alone
                    # otherwise, and its peers would wait in engine collectives it never joins
                    failed = float(self.ctrl_all_reduce([0.0 if self.xgmi is not None else 1.0],
                                                        dist.ReduceOp.MAX)[0])
                    if failed and self.xgmi is not None:
                        self.xgmi.close()
                        self.xgmi = None
                        self.xgmi_probe = {"selected": "rccl", "error": "a peer's xGMI engine failed"}
            if self.data_kind == "gloo":
                self.data = dist.ProcessGroupGloo(dist.PrefixStore("data", base), rank, world_size, _td(timeout_s))
            else:
                opts = dist.ProcessGroupNCCL.Options()
                opts.is_high_priority_stream = high_priority
                opts._timeout = _td(timeout_s)
                self.nonblocking = _rccl_nonblocking(opts, reformed=probe != "now")
                self.data = dist.ProcessGroupNCCL(dist.PrefixStore("data", base), rank, world_size, opts)
                if self.nonblocking:
                    # ncclCommInitRankConfig with blocking = 0, started now: the bootstrap runs while
                    # the epoch entry goes on (state sync over the control plane, the engine's
                    # mappings), the first collective waits for it, and abort() -- the watchdog's,
                    # when a peer dies during the bootstrap -- can end an init still in progress
                    # (non-blocking init + async error + abort)
                    try:
                        self.data.eager_connect_single_device(self.device)
                    except Exception as e:  # noqa: BLE001 - lazy init at the first collective instead
                        log.debug("eager RCCL connect failed: %s", e)
            self.backend = self.data_kind + ("+xgmi" if self.xgmi_mode == "xgmi" else "")
        else:
            self.data = dist.ProcessGroupGloo(dist.PrefixStore("data", base), rank, world_size, _td(timeout_s))
            self.backend = "gloo"
            self.data_kind = "gloo"
        self.init_s = time.perf_counter() - t0

    # -- lifecycle -----------------------------------------------------------
    def _sync_stream(self) -> None:
        """Host-wait for this rank's compute stream, which every collective is ordered
        into.  Never torch.cuda.synchronize(): that also waits for an in-flight snapshot
        copy on the checkpoint engine's stream, on the recovery path."""
        if self.device.type == "cuda":
            torch.cuda.current_stream(self.device).synchronize()

    def warmup(self) -> float:
        """Force lazy communicator creation now (so it is not hidden in step 1)."""
        t0 = time.perf_counter()
        if self.backend == "xgmi":
            self.xgmi.all_reduce(torch.zeros(64, device=self.device))
            self._sync_stream()
        elif self.data is not None:
            x = torch.zeros(1, device=self.device)
            self.data.allreduce([x]).wait()
            if self.device.type == "cuda":
                self._sync_stream()
        self.ctrl.allreduce([torch.zeros(1)]).wait()
        if self.xgmi is not None and self.xgmi_mode == "auto":
            self._select_policy()
        return time.perf_counter() - t0

    # -- all-reduce policy: cache, probe, deferral ------------------------------------
    def _policy_key(self) -> str:
        """Cache key of the agreed policy: one per (job, group, world size, ranks per GPU)
        -- the probe's answer depends on nothing else that a re-formation can change."""
        rpd = int(getattr(self.xgmi, "ranks_per_device", 1) or 1)
        return f"edl/{self._job}/commpolicy/{self.group}/w{self.world_size}/rpd{rpd}"

    def _cached_policy(self) -> dict | None:
        """The cached probe document, if EVERY rank read the same one (agreed over the
        control plane by its checksum), else None."""
        import json
        import zlib
        doc, raw = None, b""
        try:
            if self._root_store.check([self._policy_key()]):
                raw = self._root_store.get(self._policy_key())
                doc = json.loads(raw.decode())
        except Exception as e:  # noqa: BLE001 - a broken cache entry means "probe"
            log.debug("policy cache read failed: %s", e)
            doc, raw = None, b""
        crc = float(zlib.crc32(raw) if doc else -1)
        v = self.ctrl_all_reduce([crc, -crc], dist.ReduceOp.MAX)
        return doc if (doc is not None and v[0] == -v[1] and v[0] >= 0) else None

    def _store_policy(self) -> None:
        import json
        if self.rank == 0 and self.xgmi_probe and self.xgmi_probe.get("exact_everywhere") is not None \
                and "error" not in self.xgmi_probe:
            try:
                self._root_store.set(self._policy_key(), json.dumps(self.xgmi_probe))
            except Exception as e:  # noqa: BLE001 - the cache is an optimisation
                log.debug("policy cache write failed: %s", e)

    def _select_policy(self) -> None:
        """warmup() in "auto": adopt the cached policy of this (group, world) if every rank
        has it; otherwise probe now (a job's first epoch) or defer the probe until after
        the epoch's first committed step (re-formations: the probe is ~1 s of collectives
        that would otherwise sit between a fault and the first recovered step)."""
        cached = self._cached_policy()
        if cached is not None:
            # an earlier epoch's timings, but THIS epoch's mappings: they must sum exactly first
            exact = self._exact_gate()
            self._adopt_probe(dict(cached, cached=True, epoch=self.epoch, measured_epoch=cached.get("epoch"),
                                   exact_everywhere=bool(cached.get("exact_everywhere")) and exact,
                                   gate_exact=exact))
            return
        if self.probe_mode == "defer":
            self.probe_pending = True     # RCCL only until run_deferred_probe() / adopt_policy()
            return
        self._probe_xgmi()
        self._store_policy()

    def run_deferred_probe(self) -> float:
        """The deferred probe, at an agreed point (every rank after the same committed
        step).  Returns its seconds; the caller re-registers its gradient buffers if the
        engine was kept."""
        if not self.probe_pending or self.xgmi is None or self.xgmi_mode != "auto":
            self.probe_pending = False
            return 0.0
        t0 = time.perf_counter()
        self.probe_pending = False
        self._probe_xgmi()
        self._store_policy()
        return time.perf_counter() - t0

    def adopt_policy(self, pol: dict) -> bool:
        """A policy for this world size from elsewhere (the Brain's median of earlier
        epochs' probes) replaces a pending probe.  Agreed by the caller (every rank adopts
        the same runtime plan at the same point)."""
        if self.xgmi is None or self.xgmi_mode != "auto" or not self.probe_pending:
            return self.apply_allreduce_policy(pol)
        self.probe_pending = False
        exact = self._exact_gate()
        self._adopt_probe({"epoch": self.epoch, "world": self.world_size, "exact_everywhere": exact, "policy": pol,
                           "source": "brain", "gate_exact": exact})
        return self.xgmi is not None

    GATE_ELEMS = 1 << 17      # 256 KB of bf16: both engine forms that run on the workspace

    def _exact_gate(self) -> bool:
        """Correctness gate for a policy adopted without a probe (cached, or the Brain's):
        one integer-valued all-reduce through the data plane and through the engine's
        two-shot and one-shot forms on this epoch's freshly mapped workspaces, compared
        exactly on every rank and agreed (MAX of failures) over the control plane.  The
        timing sweep is what a cached policy skips; this check is not."""
        g = torch.Generator(device="cpu").manual_seed(11 + self.rank)
        src = torch.randint(-4, 5, (self.GATE_ELEMS,), generator=g, dtype=torch.int8).to(self.device, torch.bfloat16)
        bad = 0.0
        keep_timeout, self.xgmi.timeout_s = self.xgmi.timeout_s, 5.0
        try:
            ref = src.clone()
            self.data.allreduce([ref]).wait()
            for algo in ("twoshot", "oneshot"):
                t = src.clone()
                self.xgmi.all_reduce(t, algo)
                self._sync_stream()
                if not torch.equal(ref, t) or self.xgmi.status() != 0:
                    bad = 1.0
        except Exception as e:  # noqa: BLE001
            log.warning("xGMI exactness gate failed: %s", e)
            bad = 1.0
        finally:
            self.xgmi.timeout_s = keep_timeout
        bad = float(self.ctrl_all_reduce([bad], dist.ReduceOp.MAX)[0])
        if bad:
            log.warning("epoch %d: the xGMI engine did not sum exactly; all-reduce stays on %s", self.epoch,
                        self.data_kind)
        return not bad

    def _adopt_probe(self, probe: dict) -> None:
        pol = probe.get("policy") or {}
        keep = bool(probe.get("exact_everywhere")) and (pol.get("xgmi_min_kb_inplace") is not None
                                                        or pol.get("xgmi_min_kb_staged") is not None)
        probe["selected"] = "xgmi" if keep else "rccl"
        self.xgmi_probe = probe
        if keep:
            self.xgmi_mode = "xgmi"
            self.backend = self.data_kind + "+xgmi"
            self.apply_allreduce_policy(pol)
        else:
            self._sync_stream()
            self.xgmi.close()
            self.xgmi = None
            self.xgmi_mode = None

    PROBE_KB = (256, 1024, 4096, 32768, 131072)
    ONESHOT_PROBE_KB = 4096     # one-shot is timed up to this size (it reads N x S per rank)

    def _probe_xgmi(self, sizes_mb=None, iters: int = 3) -> None:
        """Measure the xGMI engine against RCCL on THIS node from latency-bound to
        gradient-bucket sizes, in each of its forms (one-shot; two-shot in place on a
        registered buffer; two-shot staged through the workspace for buffers too large
        to map), on integer-valued data so every sum is exact.  The engine is timed in
        the form training runs it: ``all_reduce_async`` on its own stream with
        ``async_blocks`` workgroups (what ElasticDDP's bucket all-reduces use under the
        backward), not the full-chip synchronous grid.  The engine is kept only if every
        rank saw an exact result; the policy (one-shot switch sizes, the size from which
        each form beats RCCL) comes from :func:`comm_policy.decide` on the per-size MAX
        over ranks, so every rank derives the same policy."""
        from easydl_amd.parallel import comm_policy
        t_probe = time.perf_counter()
        sizes_kb = tuple(int(m * 1024) for m in sizes_mb) if sizes_mb else self.PROBE_KB
        nel = (max(sizes_kb) << 10) // 2
        g = torch.Generator(device="cpu").manual_seed(7 + self.rank)
        src = torch.randint(-4, 5, (nel,), generator=g, dtype=torch.int8).to(self.device, torch.bfloat16)
        a, b = src.clone(), src.clone()
        reg = None
        keep_timeout, self.xgmi.timeout_s = self.xgmi.timeout_s, 5.0  # a broken path gives up fast
        blocks = getattr(self.xgmi, "async_blocks", None)
        # every decision point is agreed over the control plane, so a rank whose engine
        # fails locally never leaves its peers waiting inside a data-plane collective
        try:
            reg = self.xgmi.register(b)
            bad = 0.0
        except Exception as e:  # noqa: BLE001
            log.warning("xGMI probe: registration failed: %s", e)
            bad = 1.0
        bad = float(self.ctrl_all_reduce([bad], dist.ReduceOp.MAX)[0])

        def engine(algo):   # the training form: async on the engine stream, caller waits on its event
            def run(t):
                w = self.xgmi.all_reduce_async(t, algo) if blocks is not None else None
                if w is None:
                    self.xgmi.all_reduce(t, algo)
                else:
                    w.wait()
            return run
        if not bad:
            try:
                self.data.allreduce([a]).wait()
                engine(None)(b)
                self._sync_stream()
                bad = 0.0 if (torch.equal(a, b) and self.xgmi.status() == 0) else 1.0
            except Exception as e:  # noqa: BLE001
                log.warning("xGMI probe: exactness check failed: %s", e)
                bad = 1.0
            bad = float(self.ctrl_all_reduce([bad], dist.ReduceOp.MAX)[0])
        inf = float("inf")
        n = len(sizes_kb)
        cols = [[inf] * n for _ in range(4)]     # rccl, in place, staged, one-shot (seconds)
        if not bad:
            def timed(fn, t, it):
                fn(t)
                self._sync_stream()
                t0 = time.perf_counter()
                for _ in range(it):
                    fn(t)
                self._sync_stream()
                return (time.perf_counter() - t0) / it

            forms = (lambda t: self.data.allreduce([t]).wait(),
                     engine("inplace"), engine("twoshot"), engine("oneshot"))
            for i, kb in enumerate(sizes_kb):
                view = b[:(kb << 10) // 2]
                it = iters if kb > 1024 else 4 * iters      # latency-bound sizes: more samples
                failed = 0.0
                for c, fn in enumerate(forms):
                    if c == 3 and kb > self.ONESHOT_PROBE_KB:
                        continue
                    try:
                        cols[c][i] = timed(fn, view, it)
                    except Exception as e:  # noqa: BLE001
                        log.warning("xGMI probe: form %d at %d KB failed: %s", c, kb, e)
                        failed = 1.0
                        break   # the rest of this size would meet peers out of step
                try:
                    failed = max(failed, 0.0 if self.xgmi.status() == 0 else 1.0)
                except Exception:  # noqa: BLE001
                    failed = 1.0
                # agreed after every size: one rank's failure ends the probe on all ranks
                if float(self.ctrl_all_reduce([failed], dist.ReduceOp.MAX)[0]):
                    bad = 1.0
                    break
            try:
                bad = max(bad, 0.0 if self.xgmi.status() == 0 else 1.0)
            except Exception:  # noqa: BLE001
                bad = 1.0
        self.xgmi.timeout_s = keep_timeout
        big = 1e9    # inf does not travel through the control plane's tensors cleanly
        flat = [bad] + [min(v, big) for col in cols for v in col]
        worst = self.ctrl_all_reduce(flat, dist.ReduceOp.MAX)
        exact = worst[0] == 0
        cols = [[inf if float(v) >= big else float(v) for v in worst[1 + c * n:1 + (c + 1) * n]] for c in range(4)]
        pol = (comm_policy.decide(sizes_kb, *cols, world=self.world_size) if exact
               else {"oneshot_max_kb": None, "oneshot_max_staged_kb": None, "xgmi_min_kb_inplace": None,
                     "xgmi_min_kb_staged": None, "bucket_floor_mb": None, "busbw_gbs": []})
        keep = exact and (pol["xgmi_min_kb_inplace"] is not None or pol["xgmi_min_kb_staged"] is not None)
        ms = lambda col: [round(v * 1e3, 4) if math.isfinite(v) else None for v in col] if exact else []  # noqa: E731
        bw = lambda col: [round(comm_policy.busbw_gbs(k, v, self.world_size), 1)  # noqa: E731
                          for k, v in zip(sizes_kb, col)] if exact else []
        mb = lambda kb: None if kb is None else kb / 1024.0  # noqa: E731
        self.xgmi_probe = {
            "epoch": self.epoch, "world": self.world_size,
            "sizes_kb": list(sizes_kb) if exact else [], "sizes_mb": [k / 1024.0 for k in sizes_kb] if exact else [],
            "rccl_ms": ms(cols[0]), "xgmi_inplace_ms": ms(cols[1]), "xgmi_staged_ms": ms(cols[2]),
            "xgmi_oneshot_ms": ms(cols[3]),
            "rccl_busbw_gbs": bw(cols[0]), "xgmi_inplace_busbw_gbs": bw(cols[1]), "xgmi_staged_busbw_gbs": bw(cols[2]),
            "exact_everywhere": bool(exact), "policy": pol,
            "xgmi_min_mb_inplace": mb(pol["xgmi_min_kb_inplace"]), "xgmi_min_mb_staged": mb(pol["xgmi_min_kb_staged"]),
            # the engine configuration that was timed (= the one DDP buckets run)
            "engine_form": "async" if blocks is not None else "sync", "engine_blocks": blocks,
            "data_plane": self.data_kind, "probe_s": round(time.perf_counter() - t_probe, 4),
            "selected": "xgmi" if keep else "rccl"}
        log.info("all-reduce probe (epoch %d, world %d): %s", self.epoch, self.world_size, self.xgmi_probe)
        if reg is not None:
            self._sync_stream()
            self.xgmi.unregister(reg)
        self._adopt_probe(self.xgmi_probe)

    def apply_allreduce_policy(self, pol: dict) -> bool:
        """Switch the per-size routing (RCCL / engine form) to ``pol`` (see
        :func:`comm_policy.decide`).  Every rank must apply the same policy before the
        same collective: callers switch at an agreed point (the probe's control-plane
        agreement, or a committed step for the Brain's runtime plan)."""
        if self.xgmi is None or self.xgmi_mode != "xgmi":
            return False
        never = 1 << 62
        kb = lambda k: never if k is None else int(k) << 10  # noqa: E731
        self.xgmi_min_bytes = kb(pol.get("xgmi_min_kb_inplace"))
        self.xgmi_min_bytes_staged = kb(pol.get("xgmi_min_kb_staged"))
        if pol.get("oneshot_max_kb") is not None:
            self.xgmi.oneshot_max = int(pol["oneshot_max_kb"]) << 10
        if pol.get("oneshot_max_staged_kb") is not None:
            self.xgmi.oneshot_max_staged = int(pol["oneshot_max_staged_kb"]) << 10
        self.allreduce_policy = dict(pol)
        return True

    def register_buffers(self, tensors) -> None:
        """Long-lived buffers every rank registers in the same order (ElasticDDP's flat
        gradient groups): the engine then all-reduces their slices in place."""
        if self.xgmi is None or self.xgmi_mode != "xgmi":
            return
        if self.xgmi_min_bytes >= 1 << 62:
            # the (agreed) policy never routes a registered buffer to the engine: no mappings
            return
        from easydl_amd.parallel.xgmi import XgmiError
        for t in tensors:   # sizes are equal on every rank, so every rank skips the same ones
            if self.xgmi._find_registered(t)[0] is not None:
                continue    # already mapped this epoch (re-binding after a policy switch)
            if self.xgmi.supports(t) and self.xgmi.registrable(t):
                try:
                    self.xgmi.register(t)
                except XgmiError as e:   # agreed on every rank (segment too large): staged path
                    log.info("gradient buffer not registered: %s", e)

    def transfer_state(self, tensors, holders) -> None:
        """State transfer to joiners / replacements: every rank not in ``holders``
        receives each tensor, slice k from holder k, all holders sending at once over
        distinct links (SURVEY.md §2.8 "multi-source scatter").  Holders are identical
        by construction (same committed step).  Collective."""
        holders = sorted(set(int(h) for h in holders))
        if self._aborted:
            raise CommAborted("communicator aborted")
        if not holders:
            raise ValueError("transfer_state: no holder")
        if len(holders) == self.world_size:
            return
        if len(holders) == 1:   # one source: the collective broadcast is already link-optimal
            for t in tensors:
                self.broadcast(t, holders[0])
            return
        if self.xgmi is not None and self.device.type == "cuda":
            big = [t for t in tensors if self.xgmi.pullable(t)]
            rest = [t for t in tensors if not self.xgmi.pullable(t)]
            if big:
                self._native(self.xgmi.pull, big, holders)
                if self.xgmi.status() != 0:
                    raise CommAborted(f"xGMI state transfer gave up in epoch {self.epoch}: "
                                      f"{self.xgmi.status_detail()}")
            for t in rest:
                self.broadcast(t, holders[0])
            return
        receivers = [r for r in range(self.world_size) if r not in holders]
        me_holds = self.rank in holders
        ops = []   # (kind, tensor slice, peer, tag)
        for ti, t in enumerate(tensors):
            flat = t.reshape(-1)
            n = flat.numel()
            nh = len(holders)
            per = -(-n // nh)
            for k, h in enumerate(holders):
                sl = flat[k * per:min(n, (k + 1) * per)]
                if sl.numel() == 0:
                    continue
                if me_holds and self.rank == h:
                    ops += [("send", sl, r, ti) for r in receivers]
                elif not me_holds:
                    ops.append(("recv", sl, h, ti))
        if not ops:
            self._p2p_batch([])   # still take part in the group call on RCCL
            return
        self._p2p_batch(ops)

    def _p2p_batch(self, ops) -> None:
        """Concurrent point-to-point transfers (one grouped launch on RCCL)."""
        if not ops:
            return
        if self.data_kind == "rccl" and hasattr(self.data, "_start_coalescing"):
            # ProcessGroupNCCL's coalescing window (torch 2.10: no arguments): every send and
            # receive below becomes one grouped RCCL launch, so no pairing order can deadlock
            self.data._start_coalescing()
            for kind, t, peer, tag in ops:
                (self.data.send if kind == "send" else self.data.recv)([t], peer, tag)
            self._wait(self.data._end_coalescing())
            return
        # gloo: every transfer in flight at once; (peer, tag) pairs match sends to receives
        works = [(self.data.send if kind == "send" else self.data.recv)([t], peer, tag) for kind, t, peer, tag in ops]
        for w in works:
            self._wait(w)

    def healthy(self) -> bool:
        """False if a hand-written collective gave up (abort word / deadline) since the
        epoch started; read after the step's host sync, so it costs one 4-byte copy."""
        return self.xgmi is None or self.xgmi.status() == 0

    def abort(self) -> None:
        """Abort in-flight collectives (callable from a watchdog thread)."""
        with self._lock:
            if self._aborted:
                return
            self._aborted = True
        # RCCL: ncclCommAbort makes kernels blocked on a dead peer exit.  Gloo
        # collectives already fail as soon as a peer's sockets close, and
        # ProcessGroupGloo.abort() leaves worker threads that std::terminate the
        # process at teardown, so gloo groups are only marked, never aborted.
        if self.xgmi is not None:
            self.xgmi.abort()  # host-mapped abort word: spinning workgroups exit
        if self.data_kind == "rccl":
            try:
                self.data.abort()
            except Exception as e:  # pragma: no cover - best effort
                log.debug("abort failed: %s", e)

    @property
    def aborted(self) -> bool:
        return self._aborted

    def shutdown(self) -> None:
        if self._aborted:
            return
        if self.xgmi is not None:
            self.xgmi.close()
            self.xgmi = None
        for pg in (self.data, self.ctrl):
            if pg is None:
                continue
            try:
                if hasattr(pg, "shutdown"):
                    pg.shutdown()
            except Exception:
                pass

    # -- data plane ------------------------------------------------------------
    def _verify(self, kind: str, t: torch.Tensor, extra: int = 0) -> None:
        """Agree on (sequence number, signature) over the CPU control plane before the call."""
        if not self.check or self.world_size == 1:
            return
        self._seq += 1
        sig = float(_signature(kind, t, extra))
        v = self.ctrl_all_reduce([sig, -sig, float(self._seq), -float(self._seq)], dist.ReduceOp.MAX)
        if v[0] != -v[1] or v[2] != -v[3]:
            raise CollectiveMismatch(
                f"rank {self.rank} epoch {self.epoch}: collective #{self._seq} {kind}(numel={t.numel()}, "
                f"{t.dtype}) differs across ranks (signatures {int(v[0])}..{int(-v[1])})")

    def all_reduce_async(self, t: torch.Tensor, op=dist.ReduceOp.SUM):
        if self._aborted:
            raise CommAborted("communicator aborted")
        self._verify("all_reduce", t, int(op))
        if self._use_xgmi_allreduce(t):
            if op == dist.ReduceOp.SUM:
                return self._native(self.xgmi.all_reduce_async, t)
            if op == dist.ReduceOp.MAX:
                return self._native(self._xgmi_sync, self.xgmi.all_reduce_max, t)
        if self.backend == "xgmi":
            return self._xgmi_only_fallback(t, op)
        o = dist.AllreduceOptions()
        o.reduceOp = op
        return self.data.allreduce([t], o)

    def all_reduce(self, t: torch.Tensor, op=dist.ReduceOp.SUM) -> torch.Tensor:
        self._wait(self.all_reduce_async(t, op), poll=True)
        return t

    def broadcast(self, t: torch.Tensor, src: int) -> torch.Tensor:
        if self._aborted:
            raise CommAborted("communicator aborted")
        self._verify("broadcast", t, src)
        if self.backend == "xgmi":
            if self._use_xgmi(t):
                if self.rank != src:
                    t.zero_()
                self._native(self.xgmi.all_reduce, t)   # x + 0 + ... + 0 == x exactly
                torch.cuda.current_stream(self.device).synchronize()
                if self.xgmi.status() != 0:
                    raise CommAborted(f"xGMI broadcast gave up in epoch {self.epoch}")
                return t
            h = t.detach().cpu().contiguous()
            o = dist.BroadcastOptions()
            o.rootRank = src
            self._wait(self.ctrl.broadcast([h], o), poll=True)
            t.copy_(h)
            return t
        o = dist.BroadcastOptions()
        o.rootRank = src
        self._wait(self.data.broadcast([t], o), poll=True)
        return t

    def _xgmi_only_fallback(self, t: torch.Tensor, op):
        """xgmi-only data plane, tensor the engine cannot take: pad fp32/bf16 to 16 bytes,
        anything else through the CPU control plane."""
        if t.dtype in (torch.float32, torch.bfloat16) and t.is_contiguous() and op == dist.ReduceOp.SUM:
            n = t.numel()
            per = 16 // t.element_size()
            tmp = torch.zeros(-(-n // per) * per, dtype=t.dtype, device=t.device)
            tmp[:n].copy_(t.view(-1))
            self._native(self.xgmi.all_reduce, tmp)
            t.view(-1).copy_(tmp[:n])
            return _DoneWork()
        h = t.detach().cpu().contiguous()
        o = dist.AllreduceOptions()
        o.reduceOp = op
        self._wait(self.ctrl.allreduce([h], o), poll=True)
        t.copy_(h)
        return _DoneWork()

    def _use_xgmi(self, *ts) -> bool:
        return self.xgmi is not None and self.xgmi_mode == "xgmi" and all(self.xgmi.supports(t) for t in ts)

    def _use_xgmi_allreduce(self, t) -> bool:
        if not self._use_xgmi(t):
            return False
        if self.backend == "xgmi":
            return True
        nbytes = t.numel() * t.element_size()
        reg, _ = self.xgmi._find_registered(t)
        return nbytes >= (self.xgmi_min_bytes if reg is not None else self.xgmi_min_bytes_staged)

    def _xgmi_sync(self, fn, *args):
        """Run an xGMI collective on the caller's stream (TP/SP: the consumer is next)."""
        fn(*args)
        return _DoneWork()

    def all_gather_into(self, out: torch.Tensor, inp: torch.Tensor) -> torch.Tensor:
        if self._use_xgmi(out, inp):
            self._native(self.xgmi.all_gather, out, inp)
            return out
        self._wait(self.data._allgather_base(out, inp))
        return out

    def reduce_scatter_into(self, out: torch.Tensor, inp: torch.Tensor, op=dist.ReduceOp.SUM) -> torch.Tensor:
        if op == dist.ReduceOp.SUM and self._use_xgmi(out, inp):
            self._native(self.xgmi.reduce_scatter, out, inp)
            return out
        o = dist.ReduceScatterOptions()
        o.reduceOp = op
        self._wait(self.data._reduce_scatter_base(out, inp, o))
        return out

    def all_to_all_single(self, out: torch.Tensor, inp: torch.Tensor):
        self._wait(self.data.alltoall_base(out, inp, [], [], dist.AllToAllOptions()))
        return out

    def send(self, t: torch.Tensor, dst: int, tag: int = 0):
        self._wait(self.data.send([t], dst, tag))

    def recv(self, t: torch.Tensor, src: int, tag: int = 0):
        self._wait(self.data.recv([t], src, tag))
        return t

    def _native(self, fn, *args):
        try:
            return fn(*args)
        except RuntimeError as e:
            raise CommAborted(f"xGMI engine call failed in epoch {self.epoch}: {e}") from e

    def wait_work(self, work) -> None:
        """Wait for an all-reduce work object (DDP buckets): abortable on gloo."""
        self._wait(work, poll=True)

    def _wait(self, work, poll: bool = False) -> None:
        # poll only for collectives whose gloo work progresses on its own thread
        # (allreduce / broadcast / allgather); gloo's _reduce_scatter_base runs inside
        # wait() and would never report completion to a poller
        if poll and self.data_kind == "gloo":
            # gloo collectives cannot be aborted; a rank blocked on a dead peer would sit in
            # wait() until gloo's own error path unwinds the ring (~1.5 s measured).  Poll
            # instead, so the watchdog's abort() releases this rank at once (the abandoned
            # work object fails on its own when the old group's sockets close).
            while not work.is_completed():
                if self._aborted:
                    raise CommAborted(f"epoch {self.epoch} aborted while waiting for a collective")
                time.sleep(0.0002)
        try:
            work.wait()
        except Exception as e:
            raise CommAborted(f"collective failed in epoch {self.epoch}: {e}") from e
        if self._aborted:
            raise CommAborted("communicator aborted")

    # -- control plane (CPU) ---------------------------------------------------
    def ctrl_all_reduce(self, values, op=dist.ReduceOp.SUM) -> torch.Tensor:
        t = torch.as_tensor(values, dtype=torch.float64).clone().reshape(-1)
        o = dist.AllreduceOptions()
        o.reduceOp = op
        self._wait(self.ctrl.allreduce([t], o), poll=True)
        return t

    def ctrl_broadcast(self, values, src: int) -> torch.Tensor:
        t = torch.as_tensor(values, dtype=torch.float64).clone().reshape(-1)
        o = dist.BroadcastOptions()
        o.rootRank = src
        self._wait(self.ctrl.broadcast([t], o))
        return t

    def barrier(self) -> None:
        self._wait(self.ctrl.barrier())


class MeshComm:
    """One rank's communicators for a DP x TP epoch (Megatron ordering: the TP
    group is ``tp`` consecutive ranks, the DP group the ranks with equal
    ``rank % tp``).

    ``world`` carries only the control plane (agreement, barriers); gradients
    are all-reduced over ``dp``, activations over ``tp``.  On one node every
    group is fully xGMI-connected, so consecutive-rank TP needs no topology
    search; across nodes it keeps TP traffic inside a node.  ``abort()`` aborts
    all three so no rank stays blocked in any of them.
    """

    def __init__(self, world, tp, dp, tp_size: int):
        self.world, self.tp, self.dp = world, tp, dp
        self.tp_size = tp_size
        self.rank, self.world_size, self.epoch = world.rank, world.world_size, world.epoch
        self.device = world.device
        self.backend = getattr(dp, "backend", "local")
        self.init_s = sum(getattr(c, "init_s", 0.0) for c in (world, tp, dp))

    @property
    def tp_rank(self) -> int:
        return self.rank % self.tp_size

    @property
    def dp_rank(self) -> int:
        return self.rank // self.tp_size

    @property
    def aborted(self) -> bool:
        return any(c.aborted for c in (self.world, self.tp, self.dp))

    def abort(self) -> None:
        for c in (self.dp, self.tp, self.world):
            c.abort()

    def healthy(self) -> bool:
        return all(c.healthy() for c in (self.world, self.tp, self.dp))

    def shutdown(self) -> None:
        for c in (self.dp, self.tp, self.world):
            c.shutdown()

    def warmup(self) -> float:
        return sum(c.warmup() for c in (self.world, self.tp, self.dp))

    def ctrl_all_reduce(self, values, op=dist.ReduceOp.SUM):
        return self.world.ctrl_all_reduce(values, op)

    def ctrl_broadcast(self, values, src: int):
        return self.world.ctrl_broadcast(values, src)

    def barrier(self) -> None:
        self.world.barrier()


def build_mesh(store, rank: int, world: int, epoch: int, tp: int, *, device, job: str, **kw) -> MeshComm:
    """World control plane + this rank's TP and DP groups for one epoch."""
    if world % tp:
        raise ValueError(f"world {world} is not a multiple of tp={tp}")
    dp_rank, tp_rank = divmod(rank, tp)
    w = Communicator(store, rank, world, epoch, device=device, job=job, data=False, **kw)
    tpc = (Communicator(store, tp_rank, tp, epoch, device=device, job=job, tag=f"tp{dp_rank}", **kw)
           if tp > 1 else LocalCommunicator(device, epoch))
    dpn = world // tp
    dpc = (Communicator(store, dp_rank, dpn, epoch, device=device, job=job, tag=f"dp{tp_rank}", **kw)
           if dpn > 1 else LocalCommunicator(device, epoch))
    return MeshComm(w, tpc, dpc, tp)


class LocalCommunicator:
    """World of one: every collective is the identity (no process group)."""

    def __init__(self, device="cpu", epoch: int = 0):
        self.rank = 0
        self.world_size = 1
        self.epoch = epoch
        self.device = torch.device(device)
        self.backend = "local"
        self.aborted = False
        self.init_s = 0.0

    def warmup(self):
        return 0.0

    def abort(self):
        self.aborted = True

    def healthy(self):
        return True

    def shutdown(self):
        pass

    def all_reduce_async(self, t, op=None):
        return _DoneWork()

    def all_reduce(self, t, op=None):
        return t

    def broadcast(self, t, src):
        return t

    def all_gather_into(self, out, inp):
        out.copy_(inp.reshape(out.shape))
        return out

    def reduce_scatter_into(self, out, inp, op=None):
        out.copy_(inp.reshape(out.shape))
        return out

    def all_to_all_single(self, out, inp):
        out.copy_(inp)
        return out

    def ctrl_all_reduce(self, values, op=None):
        return torch.as_tensor(values, dtype=torch.float64).clone().reshape(-1)

    def ctrl_broadcast(self, values, src):
        return torch.as_tensor(values, dtype=torch.float64).clone().reshape(-1)

    def barrier(self):
        pass


class _DoneWork:
    def wait(self, *a, **k):
        return True

    def is_completed(self):
        return True
