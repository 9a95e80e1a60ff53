"""Dynamic-membership rendezvous (job-master side and worker side).

Capability: "recover failed parameter servers and workers and resume the
training" and "scale up/down the number of workers during training"
(reference README.md:25-35).  The reference gives
no mechanism; this is easydl_amd's own protocol, independent of
``torch.distributed.elastic``.

Keys (all under the job prefix of the master's TCPStore):

=========================  ===============================================
``rdzv/joined``            append-only ``node,node,...`` join log
``rdzv/info/<node>``       JSON info of a node (host, pid, local rank, gpu)
``rdzv/epoch``             counter: latest formed epoch (0 = none yet)
``rdzv/assign/<e>``        JSON ``{members, world, reason, ts}``
``rdzv/abort/<e>``         set when epoch e is broken (member died/hung)
``rdzv/leave/<node>``      graceful leave request (scale-down)
``hb/<node>``              heartbeat timestamp (wall clock)
``ev/dead/<node>``         death report (operator exit event / master)
``commit/<e>/<s>``         step-commit counter, ``decision/<e>/<s>`` outcome
=========================  ===============================================

Membership changes take effect at a step boundary: the step-commit protocol
(:meth:`RendezvousClient.commit`) makes every rank of an epoch agree, through
one write-once ``compare_set`` key, on (a) whether step s is applied and (b)
whether the epoch ends after it.  A step whose gradient all-reduce was cut
by a failure is dropped on every survivor; a step that completed everywhere
is applied everywhere — survivors never diverge, so a shrink needs no state
transfer at all.
"""
from __future__ import annotations

import datetime
import json
import logging
import os
import socket
import threading
import time
from dataclasses import dataclass

from easydl_amd.master.store import KV

log = logging.getLogger(__name__)


@dataclass
class RendezvousConfig:
    min_nodes: int = 1
    max_nodes: int = 8
    initial_nodes: int = 0          # first epoch waits for this many (0: min_nodes) ...
    initial_timeout_s: float = 300.0  # ... but not longer than this
    join_window_s: float = 0.5      # wait for stragglers before forming / growing an epoch
    heartbeat_timeout_s: float = 15.0
    policy: str = "shrink"          # on failure: "shrink" (continue with survivors) or "replace" (wait)
    replace_wait_s: float = 60.0    # "replace": how long to wait for a replacement before shrinking
    granule: int = 1                # world sizes are multiples of this (the TP degree)
    arrive_timeout_s: float = 30.0  # scale-up waits this long at most for processes still warming up


class JobFinished(Exception):
    """Training finished while this node waited for an epoch."""


class RendezvousManager:
    """Master-side membership state machine.  ``tick()`` is pure w.r.t. the store + clock."""

    def __init__(self, kv: KV, cfg: RendezvousConfig | None = None, clock=time.time, events=None):
        self.kv = kv
        self.cfg = cfg or RendezvousConfig()
        self.clock = clock
        self.events = events  # optional EventLog
        self._first_wait_ts: float | None = None
        self._broken_ts: float | None = None
        self._stop = threading.Event()
        self._thread = None
        self.dead: dict[str, str] = {}
        self.target_nodes: int | None = None  # plan-driven target (Brain / JobResource)
        self.on_dead = []  # callbacks(node) run once per death (data requeue, metrics)

    # -- store views ---------------------------------------------------------
    def joined(self) -> list[str]:
        raw = self.kv.get_str("rdzv/joined", "") or ""
        out, seen = [], set()
        for n in raw.split(","):
            if n and n not in seen:
                seen.add(n)
                out.append(n)
        return out

    def epoch(self) -> int:
        return self.kv.counter("rdzv/epoch")

    def assignment(self, e: int) -> dict | None:
        return self.kv.get(f"rdzv/assign/{e}") if e > 0 else None

    def members(self) -> list[str]:
        a = self.assignment(self.epoch())
        return list(a["members"]) if a else []

    def arriving(self, joined: list[str], now: float) -> list[str]:
        """Processes that announced themselves (RendezvousClient.arriving) and are still
        warming up: not joined, not dead, announced less than arrive_timeout_s ago."""
        raw = self.kv.get_str("rdzv/arriving", "") or ""
        settled = self.__dict__.setdefault("_arrive_settled", set())
        out = []
        for n in dict.fromkeys(x for x in raw.split(",") if x):
            if n in settled:
                continue   # decided earlier: no store round trips for it on later ticks
            if n in joined or self.kv.exists(f"ev/dead/{n}") or self.kv.exists(f"ev/exit/{n}"):
                settled.add(n)   # joined already, or died while starting (supervisor exit event)
                continue
            ts = self.kv.get(f"rdzv/arrive_ts/{n}")
            if ts is not None and now - float(ts) < self.cfg.arrive_timeout_s:
                out.append(n)
            elif ts is not None:
                settled.add(n)   # announced too long ago: never counted again
        return out

    def mark_dead(self, node: str, reason: str) -> None:
        if not self.kv.exists(f"ev/dead/{node}"):
            self.kv.set(f"ev/dead/{node}", reason)
            self._event("node_dead", node=node, reason=reason)
            for cb in self.on_dead:
                try:
                    cb(node)
                except Exception as e:  # keep the master alive
                    log.warning("on_dead callback failed: %s", e)

    def _event(self, kind, **kw):
        if self.events is not None:
            self.events.emit(kind, **kw)

    # -- state machine -------------------------------------------------------
    def _dead_set(self, nodes, now) -> set[str]:
        dead = set()
        for n in nodes:
            if self.kv.exists(f"ev/dead/{n}"):
                dead.add(n)
                continue
            hb = self.kv.get(f"hb/{n}")
            if hb is not None and now - float(hb) > self.cfg.heartbeat_timeout_s:
                self.mark_dead(n, f"heartbeat timeout ({now - float(hb):.1f}s)")
                dead.add(n)
        return dead

    def tick(self) -> int | None:
        """One control iteration; returns the new epoch number if one was formed."""
        now = self.clock()
        joined = self.joined()
        dead = self._dead_set(joined, now)
        leaving = {n for n in joined if self.kv.exists(f"rdzv/leave/{n}")}
        cur = self.epoch()
        members = self.members()
        alive = [n for n in joined if n not in dead and n not in leaving]
        broken = [m for m in members if m in dead]
        # abort every recent epoch that contains a dead node: ranks may still be
        # running an older epoch (membership changes apply at step boundaries)
        for e in range(max(1, cur - 4), cur + 1):
            a = self.assignment(e)
            if not a or self.kv.exists(f"rdzv/abort/{e}"):
                continue
            bad = [m for m in a["members"] if m in dead]
            if bad:
                self.kv.set(f"rdzv/abort/{e}", json.dumps({"dead": bad, "ts": now}))
                self._event("epoch_abort", epoch=e, dead=bad)
                if e == cur:
                    self._broken_ts = now
        max_n = self.cfg.max_nodes if self.target_nodes is None else min(self.cfg.max_nodes, self.target_nodes)
        g = max(1, self.cfg.granule)
        max_n = max_n // g * g
        waiting = [n for n in alive if n not in members]
        survivors = [m for m in members if m in alive]
        reason = None
        if cur == 0:
            want = max(self.cfg.min_nodes, min(self.cfg.initial_nodes, max_n))
            if len(alive) // g * g >= max(self.cfg.min_nodes, g):
                if self._first_wait_ts is None:
                    self._first_wait_ts = now
                waited = now - self._first_wait_ts
                if len(alive) >= max_n or (waited >= self.cfg.join_window_s and
                                           (len(alive) >= want or waited >= self.cfg.initial_timeout_s)):
                    reason = "initial"
        elif broken:
            replace_ok = (self.cfg.policy == "shrink" or len(survivors) + len(waiting) >= len(members)
                          or (self._broken_ts is not None and now - self._broken_ts >= self.cfg.replace_wait_s))
            if replace_ok and (len(survivors) + len(waiting)) // g * g >= max(self.cfg.min_nodes, g):
                reason = "failure"
        elif any(m in leaving for m in members):
            if (len(survivors) + len(waiting)) // g * g >= max(self.cfg.min_nodes, g):
                reason = "leave"
        elif len(members) > max_n:
            reason = "scale_down"
        elif waiting and len(members) < max_n and min(max_n, len(members) + len(waiting)) // g * g > len(members):
            if self._first_wait_ts is None:
                self._first_wait_ts = now
            # Every re-formation pauses the running world, so joiners of one scale event
            # are admitted together: hold while announced processes are still warming up
            # (they keep their arrive_ts fresh only until arrive_timeout_s).
            coming = len(self.arriving(joined, now)) if len(members) + len(waiting) < max_n else 0
            if len(members) + len(waiting) >= max_n or (now - self._first_wait_ts >= self.cfg.join_window_s
                                                        and not coming):
                reason = "scale_up"
        else:
            self._first_wait_ts = None
        if reason is None:
            return None
        new_members = (survivors + waiting)[:max_n]
        if reason == "scale_down":
            new_members = survivors[:max_n]
        if g > 1:
            new_members = self._arrange(members, new_members if reason == "scale_down" else survivors + waiting,
                                        min(max_n, len(new_members)) // g * g)
        e = cur + 1
        self.kv.set(f"rdzv/assign/{e}", json.dumps(
            {"members": new_members, "world": len(new_members), "reason": reason, "ts": now, "prev": cur}))
        self.kv.add("rdzv/epoch", 1)
        self._first_wait_ts = None
        self._broken_ts = None
        self._event("epoch_formed", epoch=e, world=len(new_members), reason=reason, members=new_members)
        log.info("rendezvous: epoch %d formed (%s): %s", e, reason, new_members)
        return e

    def _arrange(self, prev: list[str], cand: list[str], n: int) -> list[str]:
        """TP-aware rank order for ``n`` of the candidates (survivors first).

        A survivor keeps its TP rank (``rank % granule``) whenever a slot with
        that TP rank is free, so it still holds the right parameter shard and
        only the processes that change shard (or are new) need state."""
        g = self.cfg.granule
        slots: list[str | None] = [None] * n
        rest = []
        for node in cand:
            placed = False
            if node in prev:
                for sl in range(prev.index(node) % g, n, g):
                    if slots[sl] is None:
                        slots[sl] = node
                        placed = True
                        break
            if not placed:
                rest.append(node)
        it = iter(rest)
        return [sl if sl is not None else next(it) for sl in slots]

    # -- background loop ------------------------------------------------------
    def start(self, period_s: float = 0.02) -> None:
        def loop():
            while not self._stop.is_set():
                try:
                    self.tick()
                except Exception as ex:  # store hiccup: keep the master alive
                    log.warning("rendezvous tick failed: %s", ex)
                self._stop.wait(period_s)

        self._thread = threading.Thread(target=loop, name="edl-rdzv", daemon=True)
        self._thread.start()

    def stop(self) -> None:
        self._stop.set()
        if self._thread:
            self._thread.join(timeout=2)


@dataclass
class Assignment:
    epoch: int
    rank: int
    world: int
    members: list
    reason: str


class RendezvousClient:
    """Worker side: join, heartbeat, wait for assignments, step commit."""

    def __init__(self, kv: KV, node_id: str | None = None, info: dict | None = None,
                 heartbeat_s: float = 1.0):
        self.kv = kv
        self.node_id = node_id or f"{socket.gethostname()}-{os.getpid()}"
        self.info = info or {}
        self.heartbeat_s = heartbeat_s
        self._hb_stop = threading.Event()
        self._hb = None
        self.epoch = 0
        self.plan_version = 0

    def arriving(self) -> None:
        """Announce this process before its pre-join warm-up: the master then admits it
        together with the other joiners of the same scale event (one re-formation)."""
        self.kv.set(f"rdzv/arrive_ts/{self.node_id}", str(time.time()))
        self.kv.append("rdzv/arriving", self.node_id + ",")

    def join(self) -> None:
        self.kv.set(f"rdzv/info/{self.node_id}", json.dumps(dict(self.info, pid=os.getpid(),
                                                                  host=socket.gethostname())))
        self.kv.set(f"hb/{self.node_id}", str(time.time()))
        self.kv.append("rdzv/joined", self.node_id + ",")
        if self.heartbeat_s > 0 and self._hb is None:
            self._hb = threading.Thread(target=self._heartbeat, name="edl-hb", daemon=True)
            self._hb.start()

    def _heartbeat(self):
        while not self._hb_stop.wait(self.heartbeat_s):
            try:
                self.kv.set(f"hb/{self.node_id}", str(time.time()))
            except Exception:
                return

    def stop_heartbeat(self):
        self._hb_stop.set()

    def leave(self) -> None:
        self.kv.set(f"rdzv/leave/{self.node_id}", "1")

    def latest_epoch(self) -> int:
        return self.kv.counter("rdzv/epoch")

    def aborted(self, epoch: int) -> bool:
        return self.kv.exists(f"rdzv/abort/{epoch}")

    def wait_assignment(self, after_epoch: int = 0, timeout_s: float = 600.0, poll_s: float = 0.005) -> Assignment:
        """Block until an epoch > after_epoch that includes this node is formed.

        Raises :class:`JobFinished` when training completed while this node was
        waiting (e.g. a spare worker that a TP-granular world could not use)."""
        t_end = time.monotonic() + timeout_s
        n = 0
        while time.monotonic() < t_end:
            n += 1
            if n % 20 == 1 and (self.kv.exists("train/done") or self.kv.exists("job/done")):
                raise JobFinished(self.node_id)
            e = self.latest_epoch()
            if e > after_epoch and not self.aborted(e):
                a = self.kv.get(f"rdzv/assign/{e}")
                if a and self.node_id in a["members"]:
                    self.epoch = e
                    return Assignment(e, a["members"].index(self.node_id), a["world"], a["members"], a["reason"])
                if self.kv.exists(f"ev/dead/{self.node_id}"):
                    raise RuntimeError(f"{self.node_id} was declared dead by the master")
            time.sleep(poll_s)
        raise TimeoutError(f"no rendezvous assignment after epoch {after_epoch} within {timeout_s}s")

    # -- step commit -------------------------------------------------------------
    def _decision(self, kind: str) -> str:
        # the decider also fixes the runtime-plan version every rank switches to
        return f"{kind}:{self.latest_epoch()}:{self.kv.counter('plan/version')}"

    def commit(self, epoch: int, step: int, world: int, ok: bool, timeout_s: float = 600.0,
               gc: bool = False) -> tuple[bool, int]:
        """Agree with every rank of ``epoch`` on step ``step``.

        Returns ``(apply, latest_epoch)``: apply the optimizer step iff True;
        leave the epoch after this step iff ``latest_epoch > epoch``.  The
        agreed runtime-plan version is left in ``self.plan_version``.
        """
        dkey = f"decision/{epoch}/{step}"
        known = None   # the decision, when this rank's own compare_set already returned it
        if ok:
            c = self.kv.add(f"commit/{epoch}/{step}", 1)
            if c >= world:
                known = self.kv.compare_set(dkey, "", self._decision("commit"))
        else:
            known = self.kv.compare_set(dkey, "", self._decision("abort"))
        if known:   # compare_set returns the stored value: ours, or the one that won the race
            kind, e, pv = known.split(":")
            self.plan_version = int(pv)
            if gc and step >= 2:
                self.kv.delete(f"commit/{epoch}/{step - 2}")
                self.kv.delete(f"decision/{epoch}/{step - 2}")
            return kind == "commit", int(e)
        t_end = time.monotonic() + timeout_s
        # server-side wait: the store answers the moment the decision key is written (a
        # polling loop answered 0.5-0.7 ms late, profiles/r04_commit_latency.txt); between
        # short waits the epoch's abort flag is checked, so a dead peer still breaks the wait
        slice_td = datetime.timedelta(milliseconds=20)
        while True:
            try:
                self.kv.store.wait([dkey], slice_td)
                ready = True
            except Exception:  # noqa: BLE001 - the store signals the timeout by raising
                ready = False
            if ready:
                d = self.kv.get_str(dkey)
                kind, e, pv = d.split(":")
                self.plan_version = int(pv)
                if gc and step >= 2:
                    # everyone has read decision(step-2) before anyone can decide step-1: GC
                    self.kv.delete(f"commit/{epoch}/{step - 2}")
                    self.kv.delete(f"decision/{epoch}/{step - 2}")
                return kind == "commit", int(e)
            if self.aborted(epoch):
                self.kv.compare_set(dkey, "", self._decision("abort"))
                continue
            if time.monotonic() > t_end:
                raise TimeoutError(f"commit of step {step} in epoch {epoch} timed out")
