"""Structured event timeline (JSONL) used for time-to-recover accounting.

Every process appends ``{"ts": wall, "mono": monotonic, "kind": ..., ...}``
records to ``<run_dir>/events-<proc>.jsonl``; wall-clock stamps from processes
on the same host are directly comparable, which is what the TTR breakdown
(fault -> detect -> abort -> rendezvous -> comm init -> state sync -> first
step) uses.
"""
from __future__ import annotations

import json
import os
import threading
import time


class EventLog:
    def __init__(self, path: str | None = None, proc: str = "", echo: bool = False):
        self.path = path
        self.proc = proc
        self.echo = echo
        self._lock = threading.Lock()
        self.records: list[dict] = []
        if path:
            os.makedirs(os.path.dirname(os.path.abspath(path)), exist_ok=True)

    def emit(self, kind: str, **kw) -> dict:
        rec = {"ts": time.time(), "mono": time.monotonic(), "proc": self.proc, "kind": kind}
        rec.update(kw)
        with self._lock:
            self.records.append(rec)
            if self.path:
                with open(self.path, "a") as f:
                    f.write(json.dumps(rec, default=str) + "\n")
        if self.echo:
            print(f"[event] {json.dumps(rec, default=str)}", flush=True)
        return rec

    def last(self, kind: str) -> dict | None:
        for r in reversed(self.records):
            if r["kind"] == kind:
                return r
        return None


def read_events(run_dir: str) -> list[dict]:
    out = []
    if not os.path.isdir(run_dir):
        return out
    for fn in sorted(os.listdir(run_dir)):
        if fn.startswith("events") and fn.endswith(".jsonl"):
            with open(os.path.join(run_dir, fn)) as f:
                for line in f:
                    line = line.strip()
                    if line:
                        out.append(json.loads(line))
    out.sort(key=lambda r: r["ts"])
    return out


def ttr_breakdown(events: list[dict]) -> dict | None:
    """Time-to-recover phases relative to the first injected fault.

    Recovery is complete at the first committed step of an epoch formed after
    the fault (a step finishing in the old epoch does not count)."""
    fault = next((e for e in events if e["kind"] == "fault_injected"), None)
    if fault is None:
        return None
    t0 = fault["ts"]
    after = [e for e in events if e["ts"] >= t0]

    def first(kind, pred=lambda e: True):
        return next((e for e in after if e["kind"] == kind and pred(e)), None)

    def rel(e):
        return None if e is None else round(e["ts"] - t0, 4)

    formed = first("epoch_formed")
    new_epoch = formed["epoch"] if formed else None
    in_new = (lambda e: new_epoch is not None and e.get("epoch", -1) >= new_epoch)
    done = first("step_done", in_new)
    last_before = max((e.get("step", 0) for e in events if e["kind"] == "step_done" and e["ts"] < t0), default=0)
    out = {
        "detect_s": rel(first("node_dead")),
        "abort_s": rel(first("epoch_abort")),
        "epoch_formed_s": rel(formed),
        "replacement_spawn_s": rel(first("spawn", lambda e: e.get("role") == "worker")),
        "replacement_joined_s": rel(first("joined")),
        "comm_ready_s": rel(first("comm_ready", in_new)),
        "state_synced_s": rel(first("state_synced", in_new)),
        "first_step_s": rel(done),
        "steps_lost": None if done is None else max(0, last_before + 1 - int(done.get("step", 0))),
    }
    # all-reduce policy measurements on the recovery critical path (must be none: re-formed
    # epochs adopt a cached policy or defer the probe past their first committed step)
    t_done = done["ts"] if done is not None else float("inf")
    in_window = [e for e in after if e["ts"] <= t_done]
    out["probes_in_window"] = sum(1 for e in in_window if e["kind"] == "allreduce_probe"
                                  and not e.get("cached") and e.get("source", "probe") == "probe")
    deferred = first("allreduce_probe_deferred")
    out["deferred_probe_s"] = rel(deferred)
    out["policy_cached"] = any(e["kind"] == "allreduce_probe" and e.get("cached") for e in in_window)
    out["ttr_s"] = out["first_step_s"]
    # time to regain: the job holds the pre-fault committed step count again (an HBM resume
    # or a survivor's state: at state sync; a snapshot restore: once the lost steps are redone)
    regain = next((e for e in after if in_new(e) and (
        (e["kind"] == "state_synced" and int(e.get("step", -1)) >= last_before)
        or (e["kind"] == "step_done" and int(e.get("step", 0)) >= last_before))), None)
    out["time_to_regain_s"] = rel(regain)
    out["steps_before_fault"] = last_before
    out["fault_point"] = fault.get("point")
    return out
