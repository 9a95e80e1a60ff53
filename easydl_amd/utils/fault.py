"""Fault injection: ``EDL_FAULT`` specs such as

    kill@step=5,index=1          SIGKILL this process at step 5 (role index 1 only)
    hang@step=3,index=0          SIGSTOP itself (detected by heartbeat timeout)
    exit@step=4                  clean sys.exit(3) (a crashing worker)
    nan@step=2                   poison the gradients after backward (non-finite skip path)
    delay@step=2,ms=500          sleep before the step (straggler)
    raise@step=6                 raise RuntimeError inside the step

Several specs may be joined with ``;``.  ``point`` is ``step_start`` unless the
spec says ``point=after_backward`` (``nan`` defaults to after_backward).
Every fired fault emits a ``fault_injected`` event (wall-clock t0 of TTR).
"""
from __future__ import annotations

import os
import signal
import sys
import time


class FaultSpec:
    def __init__(self, kind: str, args: dict):
        self.kind = kind
        self.step = int(args.get("step", -1))
        self.index = int(args["index"]) if "index" in args else None
        self.role = args.get("role")
        self.ms = float(args.get("ms", 0))
        self.point = args.get("point", "after_backward" if kind == "nan" else "step_start")
        self.generation = int(args.get("gen", 0))   # only this incarnation fires (replacements do not)
        self.fired = False

    @classmethod
    def parse(cls, text: str) -> list["FaultSpec"]:
        out = []
        for part in filter(None, (p.strip() for p in text.split(";"))):
            kind, _, rest = part.partition("@")
            args = {}
            for kv in filter(None, rest.split(",")):
                k, _, v = kv.partition("=")
                args[k.strip()] = v.strip()
            out.append(cls(kind.strip(), args))
        return out


class FaultInjector:
    def __init__(self, specs: list[FaultSpec], index: int = 0, role: str = "worker", events=None,
                 generation: int = 0):
        self.generation = generation
        self.specs = specs
        self.index = index
        self.role = role
        self.events = events

    @classmethod
    def from_env(cls, ctx, events=None) -> "FaultInjector":
        return cls(FaultSpec.parse(os.environ.get("EDL_FAULT", "")), ctx.index, ctx.role, events,
                   int(os.environ.get("EDL_GENERATION", 0)))

    def maybe_inject(self, point: str, step: int, trainer=None) -> None:
        for s in self.specs:
            if s.fired or s.point != point or s.step != step:
                continue
            if s.index is not None and s.index != self.index:
                continue
            if s.role is not None and s.role != self.role:
                continue
            if s.generation != self.generation:
                continue
            s.fired = True
            if self.events is not None:
                self.events.emit("fault_injected", fault=s.kind, step=step, index=self.index)
            self._fire(s, trainer)

    def _fire(self, s: FaultSpec, trainer):
        if s.kind == "kill":
            sys.stdout.flush()
            os.kill(os.getpid(), signal.SIGKILL)
        elif s.kind == "hang":
            os.kill(os.getpid(), signal.SIGSTOP)
        elif s.kind == "exit":
            os._exit(3)
        elif s.kind == "delay":
            time.sleep(s.ms / 1000.0)
        elif s.kind == "raise":
            raise RuntimeError("injected fault")
        elif s.kind == "nan":
            if trainer is not None:
                trainer.flat.groups[0].grad[0] = float("nan")
        else:
            raise ValueError(f"unknown fault kind {s.kind}")
