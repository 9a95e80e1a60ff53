"""Recovery mechanisms of the ElasticTrainer's world-1 takeover path, split out of
``trainer/elastic.py`` so that the step loop (and its world > 1 branches) reads on its own.

``ElasticTrainer`` inherits :class:`RecoveryMixin`.  Everything here serves one case: a hot
standby replaces a dead worker on the SAME GPU (reference README.md:25-29, "recover failed ...
workers and resume the training"; BASELINE.json config 3, the headline's time-to-recover):

* **VRAM hand-over** (``_publish_vram`` / ``vram_state_tensors``): every worker exports its
  persistent state buffers over IPC; the parked standby imports them, so the dead worker's
  128 GB (Llama-3-8B) are never released and re-allocated (utils/vram.py).
* **HBM resume** (``_hbm_resume_step`` / ``_maybe_restore``): when the dead worker's GPU-written
  step marks say no update was in flight, the adopted state IS the newest committed state; else
  the newest /dev/shm snapshot is restored.
* **Gradient shadows** (``_shadow_grads`` / ``_shadow_to_host`` / ``_load_host_shadow``): the
  gradients of finished micro-batches, copied under the next one, let a replacement resume a
  step mid-way.
* **Memory plan** (``_memory_plan`` / ``_pieces``, pure policy in :func:`plan_memory`): the
  replacement starts while the driver still reclaims the dead worker's activations; its first
  steps split micro-batches and recompute just enough layers to fit what is free, re-checked
  before every micro-batch.
* **Re-home** (``_maybe_rehome`` / ``_move_state``): once settled, adopted state moves into this
  process's own allocations, so the next standby can adopt it in turn.
* **Standby warm-up coordination** (``_publish_warm_spec`` / ``_warm_window``).

Unit tests: ``tests/test_recovery_cpu.py`` (memory-plan policy, micro-batch pieces),
``tests/test_hbm_resume_cpu.py`` (resume, re-home, split steps bit-exact),
``tests/test_gshadow_cpu.py``; GPU tier: ``tests/test_second_failure_gpu.py``,
``tests/test_host_shadow_gpu.py``, ``tests/test_recompute_gpu.py``.
"""
from __future__ import annotations

import logging
import math
import os
import threading
import time
import weakref

import torch

log = logging.getLogger("easydl_amd.trainer.elastic")


class _null:
    def __enter__(self):
        return self

    def __exit__(self, *a):
        return False


class RecoveryMixin:
    """World-1 takeover machinery of :class:`~easydl_amd.trainer.elastic.ElasticTrainer`."""

    def _open_marks(self) -> None:
        """Step-mark page of this worker slot (utils/stepmarks.py), with VRAM hand-over on.
        After an HBM resume the page still holds the dead worker's marks, which the post-reap
        check re-reads (ckpt/manager.py _check_marks_after_reap): this process writes its own
        only once that check has passed (the step loop calls this again after each fence).  If
        it dies before, its replacement finds marks of a writer it did not adopt from and
        restores from the snapshot."""
        from easydl_amd.utils import vram
        if self._marks is not None or not vram.enabled() or getattr(self, "kv", None) is None:
            return
        if self.checkpoint is not None and self.checkpoint.hbm_unverified():
            return
        from easydl_amd.utils.stepmarks import StepMarks
        try:
            self._marks = StepMarks(self.ctx.job, f"{self.ctx.role}{self.ctx.index}", device=self.device)
        except OSError as e:
            log.warning("step marks unavailable: %s", e)
            return
        self._settle_marks()

    def _settle_marks(self) -> None:
        """The state is settled at self.step (epoch entry: restore / transfer done)."""
        if self._marks is None:
            return
        if self.device.type == "cuda":
            torch.cuda.current_stream(self.device).synchronize()
        self._marks.set_now(self.step)

    def _publish_vram(self) -> None:
        """Export the persistent state buffers for the hot standby on this GPU (utils/vram.py):
        if this process dies, the standby builds on them instead of waiting for the driver to
        reclaim and re-allocate 128 GB (Llama-3-8B)."""
        from easydl_amd.utils import vram
        if not (vram.enabled() and self.device.type == "cuda" and getattr(self, "kv", None) is not None):
            return
        ts = self.vram_state_tensors()
        try:
            n = vram.publish(self.kv, f"{self.ctx.role}{self.ctx.index}", self.ctx.node_id, ts)
        except Exception as e:  # noqa: BLE001 - hand-over is an optimisation; training goes on
            log.warning("vram hand-over export failed: %s", e)
            return
        self.events.emit("vram_published", tensors=n, of=len(ts),
                         adopted=dict(vram.STATS, adopted_gb=round(vram.STATS["adopted_bytes"] / 2**30, 1)))

    def vram_state_tensors(self) -> dict[str, torch.Tensor]:
        """The persistent buffers a hot standby adopts (utils/vram.py names): flat weights and
        gradients, optimizer state, module buffers (BatchNorm running statistics)."""
        ts = {}
        for g in self.flat.groups:
            ts[f"flat/{g.name}/data"], ts[f"flat/{g.name}/grad"] = g.data, g.grad
        for g, st in zip(self.flat.groups, getattr(self.opt, "state", [])):
            for k, t in st.items():
                if isinstance(t, torch.Tensor) and t is not g.data:
                    ts[f"opt/{g.name}/{k}"] = t
        for k, t in getattr(self.bufs, "tensors", {}).items():
            ts[f"bufs/{k}"] = t
        ts.update(self.flat.shadow_tensors())
        return ts

    def _publish_warm_spec(self, data) -> None:
        """Tell the parked standby on this GPU what to warm up with (operator/standby.py
        warm_device): one layer of this model's width at this job's micro-batch shape, so the
        GEMM solutions, kernels and library handles of the replacement's first step are loaded
        before it is needed.  Published before this worker's first step, and the worker waits
        for that warm-up (bounded, ``EDL_WARM_WAIT_S``, default 60 s): a warm-up never runs
        beside a training step of this GPU, and it has the memory the step's activations will
        take later.  A standby that arrives later, with training running, warms up in a window
        the job master plans and every rank applies at one step (_warm_window)."""
        from easydl_amd.utils import vram
        if (self._warm_published or not vram.enabled() or self.device.type != "cuda"
                or getattr(self, "kv", None) is None):
            return
        self._warm_published = True
        from dataclasses import asdict

        from easydl_amd.models.llama import Llama
        seq = getattr(data, "seq", None)
        spec = None
        if isinstance(self.model, Llama) and self.tp == 1 and seq:
            cfg = {k: v for k, v in asdict(self.model.cfg).items() if isinstance(v, (bool, int, float))}
            cfg["n_layers"] = 1
            spec = {"model": "llama", "cfg": cfg, "batch": [self.micro_batch, int(seq)]}
        vram.publish_warm(self.kv, f"{self.ctx.role}{self.ctx.index}", spec)
        t0 = time.perf_counter()
        limit = float(os.environ.get("EDL_WARM_WAIT_S", 60))
        # a first-generation worker also waits for a standby that is still starting (it would
        # otherwise race its warm-up); a replacement never waits for the refill behind it
        first = os.environ.get("EDL_GENERATION", "0") == "0" and not vram.ADOPTED_FROM
        state = vram.standby_warm_on(self.kv, self.device.index, pending=first)
        while state is False and time.perf_counter() - t0 < limit:
            time.sleep(0.05)
            state = vram.standby_warm_on(self.kv, self.device.index, pending=first)
        if state is not None:
            self.events.emit("standby_warm_wait", s=round(time.perf_counter() - t0, 3), warm=bool(state))

    def _warm_window(self, ww: dict) -> None:
        """Runtime plan ``warm_window`` (master/main.py _grant_warm_windows): a standby that
        arrived while this job trains warms up on this rank's GPU now, between two steps --
        grant it and wait (bounded, EDL_WARM_WINDOW_S) for its warm key.  Every rank applies the
        plan at the same committed step; ranks on other GPUs go on and meet this one at the next
        collective.  A request that is gone (handled, or its standby took over) is skipped."""
        from easydl_amd.utils import vram
        name, gpu = ww.get("standby"), self.device.index
        if (self.device.type != "cuda" or gpu not in (ww.get("gpus") or []) or not name
                or (name, ww.get("id")) in self._warm_windows):
            return
        self._warm_windows.add((name, ww.get("id")))
        req = vram.read_warm_request(self.kv, name)
        if not req or req.get("id") != ww.get("id") or name not in vram.roster(self.kv):
            return
        t0 = time.perf_counter()
        self.kv.set(f"standby/warm_grant/{name}/gpu{gpu}", str(ww.get("id")))
        limit = float(os.environ.get("EDL_WARM_WINDOW_S", 60))
        next_roster = t0 + 0.5
        while not self.kv.exists(f"standby/warm/{name}/gpu{gpu}") and time.perf_counter() - t0 < limit:
            time.sleep(0.02)
            if time.perf_counter() > next_roster:     # a standby that took over or died ends the window
                next_roster = time.perf_counter() + 0.5
                if name not in vram.roster(self.kv):
                    break
        self.events.emit("standby_warm_window", standby=name, step=self.step, s=round(time.perf_counter() - t0, 3),
                         warm=self.kv.exists(f"standby/warm/{name}/gpu{gpu}"))

    def _publish_act(self) -> None:
        """HBM a step needs beyond the persistent state (activations, workspaces), after the
        first step: a replacement that adopts the state checks it against what the GPU has free
        (_memory_plan)."""
        from easydl_amd.utils import vram
        if (self._act_published or not vram.enabled() or self.device.type != "cuda"
                or getattr(self, "kv", None) is None):
            return
        if self._mb_limited:
            return      # a memory-limited step's peak is not a full step's (_memory_plan)
        self._act_published = True
        # only this process's own allocations count against its allocator's peak: state adopted
        # from a dead worker is imported memory the caching allocator never reserved (counting it
        # published 0 for a replacement, and the next replacement would not have split its step)
        adopted = set(vram.TAKEN.values())
        persistent = sum(t.untyped_storage().nbytes() for t in self.vram_state_tensors().values()
                         if t.data_ptr() not in adopted)
        act = max(0, torch.cuda.max_memory_reserved(self.device) - persistent)
        # what stays allocated between steps beyond the state (transposed-weight caches, workspaces):
        # a split micro-batch does not shrink it
        fixed = min(act, max(0, torch.cuda.memory_allocated(self.device) - persistent))
        vram.publish_act(self.kv, f"{self.ctx.role}{self.ctx.index}", act, self.micro_batch, fixed)
        self._maybe_shadow(act)

    def _maybe_shadow(self, act: int) -> None:
        """Turn the gradient shadow on after the first step if the GPU can afford it: a
        replacement starts with only the HBM this worker leaves free (the rest of its memory
        is reclaimed seconds after it dies), and its first step must still fit one sample per
        micro-batch there (_memory_plan).  At Llama-3-8B (2 x 8k tokens per micro-batch) the
        16 GB shadow does not fit that budget: the first step then blocked in hipMalloc and
        the time-to-recover doubled (profiles/r05_ttr_headline.md), so it stays off there."""
        if self.flat.gshadow is not None or not self._shadow_wanted():
            return
        from easydl_amd.utils import vram
        free = torch.cuda.mem_get_info(self.device)[0]
        if not vram.standby_warm_on(self.kv, self.device.index):
            # no warm standby on this GPU yet (a replacement before its refill arrives): keep the
            # room one will take (a context, the GEMM libraries' workspaces, its warm-up's cache)
            free -= int(float(os.environ.get("EDL_STANDBY_RESERVE_GB", "16")) * 2**30)
        shadow = sum(g.grad.untyped_storage().nbytes() for g in self.flat.groups)
        need = act / max(1, self.micro_batch) * 1.15
        mode = os.environ.get("EDL_GRAD_SHADOW", "1")
        # default: HBM where it fits, else none.  The host shadow is opt-in ("host"): at the 8B
        # headline its device -> host copies share the host link with the snapshots' (every 2
        # steps), so a kill right after a snapshot step found no finished copy, and the dead
        # worker's 30 GB of page-locked memory delayed its teardown and the replacement's first
        # step by ~0.3 s (profiles/r05_grad_shadow_ab.md)
        where = ("hbm" if mode == "force" or (mode != "host" and free - shadow >= need)
                 else "host" if mode == "host" else None)
        self.events.emit("grad_shadow", on=where is not None, where=where, gb=round(shadow / 2**30, 1),
                         free_gb=round(free / 2**30, 1), replacement_need_gb=round(need / 2**30, 1))
        if where is None:
            return
        if where == "hbm":
            self.flat.ensure_shadow(self._state_pool())
            self._publish_vram()
            return
        # host memory: the page-locked segment is created and registered off the step path; the
        # shadow copies start once it is ready
        from easydl_amd.utils.gshadow import HostShadow
        slot = f"{self.ctx.role}{self.ctx.index}"

        def make():
            t0 = time.perf_counter()
            try:
                hs = HostShadow(self.ctx.job, slot, self.flat.groups)
            except Exception as e:  # noqa: BLE001 - an optimisation: without it a step is recomputed
                self.events.emit("grad_shadow_failed", where="host", error=str(e)[:200])
                return
            self._hshadow_views = [(hs.group_views(i), hs.loss_view(i)) for i in (0, 1)]
            self._hshadow = hs
            self.events.emit("grad_shadow_ready", where="host", pinned=hs.pinned, gb=round(hs.total / 2**30, 1),
                             s=round(time.perf_counter() - t0, 3))
        threading.Thread(target=make, name="edl-gshadow", daemon=True).start()

    def _maybe_rehome(self) -> None:
        """Once a takeover's state is settled, move everything built on the dead worker's HBM into
        this process's own allocations, between two steps (FlatParams.rehome: one group at a
        time).  Imported memory cannot be exported again, so until then this process has
        nothing to hand to the next standby: a second failure of this rank would restore from
        /dev/shm instead of resuming from HBM.  Waits until the adopted state is verified (the
        post-reap step-mark check, an early hand-over's check, a deferred restore), full
        micro-batches are back and one group's copy fits in free HBM."""
        from easydl_amd.utils import vram
        if self._rehomed or not vram.adopted_any() or self.flat is None or self.opt is None:
            return
        if self.comm is None or self.comm.world_size > 1:
            # only one rank moves its buffers, and re-registering the moved gradients with the xGMI
            # engine is collective (a world-8 drill hung there); an HBM resume -- what the re-published
            # state is for -- happens at world 1 only, so the move waits for a world of one
            return
        ck = self.checkpoint
        if ck is not None and (getattr(ck, "_marks_check", None) is not None or getattr(ck, "_verify", None) is not None
                               or getattr(ck, "_deferred", None)):
            return
        if self._mb_limited:
            return
        adopted = set(vram.TAKEN.values())
        before = {k: t for k, t in self.vram_state_tensors().items() if t.data_ptr() in adopted}
        sizes = [t.untyped_storage().nbytes() for t in before.values()]
        # weak references: which buffer still is the adopted one afterwards (a freed adopted
        # range's address can come back for a new allocation, so pointers cannot tell)
        before = {k: weakref.ref(t) for k, t in before.items()}
        refs = list(before.values())

        def is_adopted(t):
            return any(r() is t for r in refs)
        if self.device.type == "cuda" and sizes and self._hbm_avail() < 2 * max(sizes):
            return
        t0 = time.perf_counter()
        self.wait_update()
        if ck is not None:
            ck.wait()           # no snapshot copy may read a buffer while it moves
        if self.device.type == "cuda":
            # the new buffers get segments of their own (fresh allocations, not blocks split out
            # of a cached activation segment): an IPC export maps a buffer's whole segment
            torch.cuda.empty_cache()
        # each moved buffer frees its adopted original as the last reference goes; should one stay
        # referenced, HBM would shrink by a buffer per move: stop while the next step's
        # activations and two buffers still fit (the rest stays on adopted memory, still correct)
        reserve = getattr(self, "_act_need", 0) + 2 * max(sizes, default=0)
        can_continue = (lambda: self._hbm_avail() >= reserve) if self.device.type == "cuda" else (lambda: True)
        n = self._move_state(is_adopted, can_continue)
        left = [k for k, t in self.vram_state_tensors().items() if k in before and before[k]() is t]
        if self.device.type == "cuda":
            torch.cuda.current_stream(self.device).synchronize()
        self._rehomed = True    # (once: a partial move is not retried)
        if left:
            for k in [k for k in vram.TAKEN if k not in left]:
                vram.TAKEN.pop(k)
            self.events.emit("rehome_partial", buffers=n, left=left[:8], n_left=len(left), step=self.step,
                             avail_gb=round(self._hbm_avail() / 2**30, 1), s=round(time.perf_counter() - t0, 3))
            return
        vram.TAKEN.clear()
        vram.ADOPTED_FROM.clear()
        self.events.emit("rehomed", buffers=n, gb=round(sum(sizes) / 2**30, 2), step=self.step,
                         s=round(time.perf_counter() - t0, 3))
        self._publish_vram()    # the next standby can adopt this state again
        for attempt in range(5):
            # a buffer whose export failed ("invalid argument": 1-8 of 95 at Llama-3-8B, where a new
            # allocation reuses an address range an imported buffer had; profiles/r05_three_failures_8b.md) moves
            # once more, to another fresh allocation, and the state is published again
            if not vram.FAILED or self.device.type != "cuda":
                break
            names = list(vram.FAILED)
            ts = self.vram_state_tensors()
            targets = [ts[k] for k in names if k in ts]
            del ts
            self._move_state(lambda t: any(t is x for x in targets))
            del targets
            torch.cuda.current_stream(self.device).synchronize()
            self.events.emit("rehome_export_retry", names=names[:8], attempt=attempt + 1)
            self._publish_vram()

    def _move_state(self, pick, can_continue=lambda: True) -> int:
        """(World 1.) Move the state buffers ``pick(tensor)`` selects to fresh allocations of this process
        (FlatParams.rehome, optim.rehome_state, FlatBuffers.rehome).  Allocated from a private
        pool: every buffer gets a segment of its own, never a block of a cached (possibly
        > 2 GiB) segment, which fails to export."""
        from easydl_amd.optim import rehome_state
        alias = [st.get("master") is not None and st["master"].data_ptr() == g.data.data_ptr()
                 for g, st in zip(self.flat.groups, self.opt.state)]
        pool = torch.cuda.use_mem_pool(self._state_pool()) if self.device.type == "cuda" else _null()
        with pool:
            n = self.flat.rehome(pick, can_continue)
            for g, st, a in zip(self.flat.groups, self.opt.state, alias):
                if a:
                    st["master"] = g.data   # an fp32 model's master IS its weight buffer
            n += rehome_state(self.opt.state, pick, can_continue)
            if self.bufs is not None:
                n += self.bufs.rehome(pick, can_continue)
        if self.ddp is not None:
            self.ddp.set_bucket_mb(self.ddp.bucket_mb)      # bucket views of the new gradient buffers
        return n

    def _state_pool(self):
        if getattr(self, "_pool", None) is None:
            self._pool = torch.cuda.MemPool()
        return self._pool

    def _hbm_avail(self) -> int:
        free, _ = torch.cuda.mem_get_info(self.device)
        return free + torch.cuda.memory_reserved(self.device) - torch.cuda.memory_allocated(self.device)

    def _memory_plan(self) -> None:
        """A replacement that adopted a dead worker's HBM starts while the driver is still
        reclaiming the rest of that worker's memory (its activations: ~82 GB for Llama-3-8B at
        2 x 8k tokens per micro-batch).  A first step that needs more than the GPU has free
        blocks inside hipMalloc until the reclaim is done -- 6 s of an 8 s time-to-recover
        (profiles/r05_ttr_headline.md).  Instead, while memory is short, each micro-batch is
        split into smaller ones: the same samples, the same loss weights, the same gradient sum
        (only the order of the bf16 additions differs), at roughly half the activation memory.
        Models with dropout are the exception: the pieces of micro-batch i are seeded once and draw
        their masks one after another, so a split step is NOT bit-exact with the unsplit one there
        (Llama, the only model this path serves, has no dropout).
        When not even one sample per piece fits, a model with a ``cfg.recompute`` knob (Llama)
        recomputes the activations of just enough of its layers in the backward
        (:func:`plan_memory`), not all of them.

        The plan follows the driver's reclaim as it happens: it is re-made before EVERY
        micro-batch (``_pieces``), so a first step that starts short of memory returns to full
        micro-batches, and drops the recompute, the moment the memory is back -- the step does
        not depend on a guess of how fast the box reclaims (5.58 s on the driver's
        box vs 3.05 s on the builder's)."""
        from easydl_amd.utils import vram
        self._restore_full_batches()
        if (self.device.type != "cuda" or self.tp > 1 or not vram.adopted_any()
                or getattr(self, "kv", None) is None or os.environ.get("EDL_RECOVERY_SPLIT", "1") == "0"):
            return
        need, mbs, fixed = vram.read_act(self.kv, f"{self.ctx.role}{self.ctx.index}")
        if not need or mbs != self.micro_batch:
            return
        self._act_need, self._act_fixed = need, fixed
        avail = self._hbm_avail()
        if avail >= need * 1.05:
            return
        self._mb_limited = True
        split, rc = self._apply_memory_plan(avail)
        self.events.emit("memory_limited_steps", step=self.step, split=split, recompute=rc > 0, recompute_layers=rc,
                         layers=self._recompute_layers_total(), need_gb=round(need / 2**30, 1),
                         avail_gb=round(avail / 2**30, 1), margin=self._memory_margin())

    @staticmethod
    def _memory_margin() -> float:
        return float(os.environ.get("EDL_RECOVERY_MARGIN", "1.15"))

    def _recompute_layers_total(self) -> int:
        """Layers whose activations the model can recompute (0: no ``cfg.recompute`` knob)."""
        cfg = getattr(self.model, "cfg", None)
        if cfg is None or not isinstance(getattr(cfg, "recompute", None), (bool, int)):
            return 0
        return int(getattr(cfg, "n_layers", 0) or 0)

    def _apply_memory_plan(self, avail: int) -> tuple[int, int]:
        """Set the split and the recomputed layer count for ``avail`` bytes of free HBM."""
        split, rc = plan_memory(self._act_need, avail, self.micro_batch, self._recompute_layers_total(),
                                self._memory_margin(), fixed=getattr(self, "_act_fixed", 0))
        self._mb_split, self._mb_plan = split, (split, rc)
        cfg = getattr(self.model, "cfg", None)
        if rc > 0:
            if self._mb_recompute is None:
                self._mb_recompute = cfg.recompute
            cfg.recompute = rc if rc < cfg.n_layers else True
        elif self._mb_recompute is not None:
            cfg.recompute, self._mb_recompute = self._mb_recompute, None
        return split, rc

    def _restore_full_batches(self) -> None:
        self._mb_split, self._mb_plan = 1, (1, 0)
        self._mb_limited = False
        if self._mb_recompute is not None:
            self.model.cfg.recompute, self._mb_recompute = self._mb_recompute, None

    def _replan_memory(self, mb: int, grow: bool = True) -> None:
        """Before micro-batch ``mb`` of a memory-limited step: full micro-batches if the memory
        is back, else the plan for what is free now.  ``grow=False`` (inside a step): the plan
        may only shrink -- pieces that grow need new, larger allocator segments, and fresh HBM
        right after the driver's reclaim costs seconds to hand out (r06 drill: a mid-step return
        to full micro-batches took 2.7 s instead of 0.7 s, profiles/r06_ttr_first_step.md)."""
        avail = self._hbm_avail()
        before = self._mb_plan
        if avail >= self._act_need * 1.05:
            if not grow:
                return
            self.events.emit("memory_restored", step=self.step, mb=mb, avail_gb=round(avail / 2**30, 1))
            self._restore_full_batches()
            return
        split, rc = plan_memory(self._act_need, avail, self.micro_batch, self._recompute_layers_total(),
                                self._memory_margin(), fixed=getattr(self, "_act_fixed", 0))
        if not grow and (split < before[0] or rc < before[1]):
            return
        split, rc = self._apply_memory_plan(avail)
        if (split, rc) != before:
            self.events.emit("memory_replanned", step=self.step, mb=mb, split=split, recompute_layers=rc,
                             avail_gb=round(avail / 2**30, 1))

    def _piece_trace_begin(self):
        """Per-piece timing of a memory-limited step (the evidence of where a takeover's first
        step goes: host time per piece is enqueue + allocator stalls, GPU time is the kernels)."""
        if not self._mb_limited or self.device.type != "cuda":
            return None
        return []

    def _piece_trace_mark(self, tr: list, mb, n: int) -> None:
        ev = torch.cuda.Event(enable_timing=True)
        ev.record(torch.cuda.current_stream(self.device))
        tr.append((mb, n, time.perf_counter(), ev, self._mb_plan, self._hbm_avail()))
        if mb is None:
            self._piece_trace = tr

    def _piece_trace_emit(self) -> None:
        """After the (drained) step: one event with every piece's host and GPU time."""
        tr, self._piece_trace = getattr(self, "_piece_trace", None), None
        if not tr or len(tr) < 2:
            return
        tr[-1][3].synchronize()
        pieces = [{"mb": a[0], "n": a[1], "host_s": round(b[2] - a[2], 4),
                   "gpu_s": round(a[3].elapsed_time(b[3]) / 1e3, 4), "split": a[4][0], "recompute": a[4][1],
                   "avail_gb": round(a[5] / 2**30, 1)} for a, b in zip(tr, tr[1:])]
        self.events.emit("limited_step_pieces", step=self.step, pieces=pieces,
                         gpu_s=round(sum(p["gpu_s"] for p in pieces), 4),
                         host_s=round(sum(p["host_s"] for p in pieces), 4))

    def _pieces(self, mbs: list):
        """(micro-batch index, sample indices, last) of a step's forward/backward passes: the
        micro-batches themselves, or -- in a memory-limited step -- their pieces, re-planned
        before every micro-batch (the pieces keep their micro-batch's index)."""
        for n, (mb, idx) in enumerate(mbs):
            if self._mb_limited:
                self._replan_memory(mb, grow=n == 0)
            k = self._mb_split
            idx = list(idx)
            step = -(-len(idx) // k) if k > 1 else max(1, len(idx))
            parts = [idx[i:i + step] for i in range(0, len(idx), step)] or [idx]
            for j, part in enumerate(parts):
                yield mb, part, n == len(mbs) - 1 and j == len(parts) - 1
                # the step-invariant part (transposed-weight caches, workspaces) is resident after
                # the first piece: later plans count only what scales with the piece
                if getattr(self, "_act_fixed", 0):
                    self._act_need = max(0, self._act_need - self._act_fixed)
                    self._act_fixed = 0

    def _hbm_resume_step(self) -> int | None:
        """Step K if this process adopted a dead worker's HBM (utils/vram.py) whose step marks
        (utils/stepmarks.py) say the update of step K had finished and none was in flight."""
        from easydl_amd.utils import stepmarks, vram
        pid = vram.ADOPTED_FROM.get("pid")
        if (pid is None or self.tp > 1 or self.comm is None or self.comm.world_size != 1
                or os.environ.get("EDL_HBM_RESUME", "1") == "0"):
            return None
        marks = stepmarks.read_slot(self.ctx.job, f"{self.ctx.role}{self.ctx.index}", shadow=True)
        if marks is None:
            return None
        begin, done, writer, *shadow = marks
        self._shadow_cand = tuple(shadow)
        if writer != pid or begin != done:
            self.events.emit("hbm_resume_refused", begin=begin, done=done, writer=writer, adopted_from=pid)
            return None
        # every tensor of the training state must be the dead worker's: one that was not
        # exported, not mapped or not taken (size / dtype / layout changed) holds init values
        from easydl_amd.ckpt.manager import CheckpointManager
        need = CheckpointManager.state_of(self) + [(f"model.{g.name}", g.data) for g in self.flat.groups]
        miss = vram.missing(need)
        if miss:
            self.events.emit("hbm_resume_refused", reason="incomplete", missing=miss[:8], n_missing=len(miss),
                             of=len(need), begin=begin, done=done)
            return None
        return done

    def _maybe_restore(self, defer_moments: bool = False) -> bool:
        """State of a process that holds none: the dead worker's HBM (HBM resume), else the
        newest snapshot.  With neither, buffers adopted from a dead worker are reset to this
        process's seeded init (a fresh start).  True if trained state was recovered."""
        t0 = time.perf_counter()
        if self.checkpoint is not None:
            k = self._hbm_resume_step()
            if k is not None:
                from easydl_amd.utils import vram
                pid = vram.ADOPTED_FROM.get("pid")
                verify = None if vram.reaped(pid) else {"pid": pid, "marks": (k, k), "job": self.ctx.job,
                                                        "slot": f"{self.ctx.role}{self.ctx.index}"}
                from easydl_amd.utils.stepmarks import best_shadow
                cand = getattr(self, "_shadow_cand", (0, 0, 0, 0))
                sh = self.flat.shadow_tensors()
                host = not sh and self._host_shadow_exists()
                best = best_shadow(cand if host else cand[:2], k + 1)   # (the HBM shadow: slot 0 only)
                if (sh or host) and best is None and any(cand[1::2]):
                    self.events.emit("grad_shadow_unused", marks=list(cand), resume_step=k)
                if best is not None and (host or not vram.missing(list(sh.items()))):
                    # the dead worker had finished best[1] micro-batches of step k + 1 (their
                    # gradients are in its shadow): that step resumes there (_run_step)
                    self._shadow_resume = {"step": k + 1, "mb": best[1], "host": host, "slot": best[0]}
                    if verify is not None:
                        verify["shadow"] = tuple(cand)
                src = self.checkpoint.resume_from_hbm(self, k, verify)
                self.events.emit("restored", step=self.step, source=src, s=round(time.perf_counter() - t0, 3))
                return True
            st = self.checkpoint.restore_latest(self, defer_moments=defer_moments)
            if st is not None:
                from easydl_amd.ckpt import manager as _ckm
                self.events.emit("restored", step=self.step, source=st, s=round(time.perf_counter() - t0, 3),
                                 h2d=dict(_ckm.LAST_RESTORE_STATS))
                return True
        self._reinit_adopted()
        return False

    def _reinit_adopted(self) -> None:
        """Nothing overwrites this process's state: buffers it built on a dead worker's HBM
        (kept for an HBM resume that did not happen) go back to the seeded init."""
        from easydl_amd.utils import vram
        if not vram.adopted_any() or self.flat is None:
            return
        n = self.flat.reinit_adopted() + (self.bufs.reinit_adopted() if self.bufs is not None else 0)
        self.opt.reset_state()
        if self.device.type == "cuda":
            torch.cuda.current_stream(self.device).synchronize()
        self.events.emit("adopted_reinit", tensors=n)

    def _host_shadow_exists(self) -> bool:
        from easydl_amd.utils.gshadow import seg_name
        return self.device.type == "cuda" and os.path.exists(
            "/dev/shm" + seg_name(self.ctx.job, f"{self.ctx.role}{self.ctx.index}"))

    def _shadow_wanted(self) -> bool:
        """Gradient shadows pay off where a replacement resumes from this process's HBM: one rank
        (HBM resume needs world 1), VRAM hand-over on, several micro-batches per step."""
        from easydl_amd.utils import vram
        return (vram.enabled() and self.device.type == "cuda" and self.tp == 1 and self.flat is not None
                and self.comm is not None and self.comm.world_size == 1 and self.global_batch is not None
                and self.global_batch > self.micro_batch and os.environ.get("EDL_GRAD_SHADOW", "1") != "0")

    def _shadow_active(self) -> bool:
        return (self._marks is not None and (self.flat.gshadow is not None or self._hshadow is not None)
                and not self._mb_limited and self.comm.world_size == 1)

    def _shadow_grads(self, mbs_done: int, loss_acc) -> None:
        """After a micro-batch's backward: copy the accumulated gradients (and the partial loss)
        into the shadow on a side stream, under the next micro-batch's forward, between an
        invalidating and a validating step mark (utils/stepmarks.py).  The next backward waits
        for the copy.  Gradients no micro-batch has written yet are zeroed first (as the end of
        the step would), so the shadow is exact."""
        self.flat.finalize_untouched()
        if self.flat.gshadow is None:
            self._shadow_to_host(mbs_done, loss_acc)
            return

        def copy(st):
            self._marks.shadow(self.step + 1, 0, st)
            with torch.no_grad():
                for g, t in zip(self.flat.groups, self.flat.gshadow):
                    t.copy_(g.grad)
                self.flat.gshadow_loss.copy_(loss_acc.reshape(1))
            self._marks.shadow(self.step + 1, mbs_done, st)
        if self.device.type != "cuda":
            copy(None)
            return
        if self._shadow_stream is None:
            from easydl_amd.utils.resources import new_stream
            self._shadow_stream = new_stream(self.device)
        st = self._shadow_stream
        st.wait_stream(torch.cuda.current_stream(self.device))
        with torch.cuda.stream(st):
            copy(st)
        loss_acc.record_stream(st)
        self._shadow_pending = True

    def _load_host_shadow(self, slot: int):
        """The dead worker's host shadow ``slot`` -> this process's gradient buffers (pipelined
        shm -> HBM copy); returns the partial loss (a 0-d CUDA tensor), None if it failed."""
        from easydl_amd.utils.gshadow import HostShadow
        t0 = time.perf_counter()
        loss = torch.zeros(1, dtype=torch.float32, device=self.device)
        stats: dict = {}
        try:
            hs = HostShadow(self.ctx.job, f"{self.ctx.role}{self.ctx.index}", self.flat.groups, create=False,
                            pin=False)
            try:
                hs.load_into(self.flat.groups, loss, slot, stats)
            finally:
                hs.close()
        except (OSError, RuntimeError) as e:
            # the whole step is recomputed instead, from zeroed gradients (a failed copy may have
            # written part of them)
            with torch.no_grad():
                for g in self.flat.groups:
                    g.grad.zero_()
            self.events.emit("grad_shadow_load_failed", where="host", error=str(e)[:200])
            return None
        self.flat.mark_accumulating()
        self.events.emit("grad_shadow_loaded", where="host", slot=slot, s=round(time.perf_counter() - t0, 3),
                         gbps=stats.get("gbps"))
        return loss[0]

    def _shadow_to_host(self, mbs_done: int, loss_acc) -> None:
        """Host gradient shadow (utils/gshadow.py): device -> host copies group by group on a side
        stream, in the order the next backward writes the groups; each parameter's next write
        waits for its group's copy only (gradsink.await_shadow), not the next micro-batch for all
        of them."""
        slot = self._hshadow_next = 1 - getattr(self, "_hshadow_next", 1)   # alternate: 0, 1, 0, ...
        views, loss_view = self._hshadow_views[slot]
        main = torch.cuda.current_stream(self.device)
        if self._shadow_stream is None:
            from easydl_amd.utils.resources import new_stream
            self._shadow_stream = new_stream(self.device)
        st = self._shadow_stream
        st.wait_stream(main)
        with torch.cuda.stream(st):
            self._marks.shadow(self.step + 1, 0, st, slot)
            for g, hv in zip(self.flat.groups, views):
                hv.copy_(g.grad.view(-1), non_blocking=True)
                ev = torch.cuda.Event()
                ev.record(st)
                for sl in g.slots:
                    sl.param._edl_wait = ev
            loss_view.copy_(loss_acc.reshape(1).float(), non_blocking=True)
            self._marks.shadow(self.step + 1, mbs_done, st, slot)
        loss_acc.record_stream(st)


def plan_memory(need: int, avail: int, mbs: int, layers: int = 0, margin: float = 1.15,
                layer_frac: float = 0.9, fixed: int = 0) -> tuple[int, int]:
    """(split, recompute_layers) for a step whose full micro-batch of ``mbs`` samples needs
    ``need`` bytes beyond the state -- ``fixed`` of them whatever the micro-batch (transposed-
    weight caches, workspaces), the rest activations that scale with it -- when ``avail`` bytes
    are free.

    * enough memory: (1, 0);
    * else the smallest split ``d`` (a divisor of ``mbs``) whose piece fits:
      ``(fixed + (need - fixed) / d) * margin <= avail``;
    * else one sample per piece, with the fewest recomputed layers that fit: recomputing ``r`` of
      ``layers`` layers frees about ``r / layers`` of the ``layer_frac`` share of a sample's
      activations that the layers hold (the rest: embedding, logits, loss).  ``layers == 0``
      (no recompute knob): (mbs, 0) and the allocator waits for the memory."""
    if avail >= need * 1.05:
        return 1, 0
    fixed = max(0, min(fixed, need))
    scaling = need - fixed
    for d in range(2, mbs + 1):
        if mbs % d == 0 and (fixed + scaling / d) * margin <= avail:
            return d, 0
    if layers <= 0:
        return mbs, 0
    sample = scaling / max(1, mbs)
    room = avail / margin - fixed          # what one sample's activations may take
    r = math.ceil(layers * (1.0 - room / sample) / layer_frac) if sample > 0 else 0
    return mbs, max(1, min(layers, r))
