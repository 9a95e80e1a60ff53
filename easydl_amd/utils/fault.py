"""Fault injection: ``EDL_FAULT`` specs such as

    kill@step=5,index=1          SIGKILL this process at step 5 (role index 1 only)
    hang@step=3,index=0          SIGSTOP itself (detected by heartbeat timeout)
    exit@step=4                  clean sys.exit(3) (a crashing worker)
    nan@step=2                   poison the gradients after backward (non-finite skip path)
    delay@step=2,ms=500          sleep before the step (straggler)
    raise@step=6                 raise RuntimeError inside the step
    kill@step=4,after_ms=1500    SIGKILL 1.5 s after step 4 starts on the GPU (mid-step; the
                                 trainer's step-start GPU event, not the host's enqueue time)
    kill@step=4,wait=standby     first step >= 4 once the hot standby on this GPU has
                                 warmed up (utils/vram.py standby_warm_on), at most 30 steps late
    kill@step=6,point=in_update  SIGKILL inside the optimizer update of step 6: after its
                                 ``begin`` step mark reached the GPU, before ``done``
    kill@step=4,point=microbatch,mb=3
                                 SIGKILL once the GPU has finished micro-batch 3 of step 4
                                 (its backward and the gradient shadow's copy), before the next;
                                 with ``after_ms``: that long after (inside micro-batch 4)

Several specs may be joined with ``;``.  ``point`` is ``step_start`` unless the
spec says ``point=after_backward`` / ``point=in_update`` (``nan`` defaults to
after_backward).  Every fired fault emits a ``fault_injected`` event (wall-clock
t0 of TTR): for a delayed fault (``after_ms``) the event is written right before
the signal, so TTR starts at the kill itself.
"""
from __future__ import annotations

import os
import signal
import sys
import threading
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
        self.after_ms = float(args.get("after_ms", 0))
        self.wait = args.get("wait")               # "standby": hold off until the spare is warm
        self.max_late = int(args.get("max_late", 30))
        self.mb = int(args.get("mb", -1))          # point=microbatch: after this micro-batch
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

    def maybe_inject(self, point: str, step: int, trainer=None, mb: int | None = None) -> None:
        for s in self.specs:
            if s.fired or s.point != point or (point == "microbatch" and s.mb != mb):
                continue
            if s.step != step and not (s.wait and s.step <= step):
                continue
            if s.index is not None and s.index != self.index:
                continue
            if s.role is not None and s.role != self.role:
                continue
            if s.generation != self.generation:
                continue
            if s.wait and step < s.step + s.max_late and not self._condition(s, trainer):
                continue
            s.fired = True
            if point in ("in_update", "microbatch") and trainer is not None \
                    and getattr(trainer, "device", None) is not None and trainer.device.type == "cuda":
                # the update's ``begin`` mark (the micro-batch's shadow copy) is written in stream
                # order: make sure it landed, so the kill is where the step marks say it is
                import torch
                torch.cuda.synchronize(trainer.device)
            if s.after_ms > 0:
                # the step runs on; the signal lands mid-step (GPU work of this step in flight),
                # ``after_ms`` after the GPU reached the step's start (the trainer's step event)
                ev = getattr(trainer, "_step_ev", None) if point == "step_start" else None
                threading.Thread(target=self._delayed, args=(s, step, trainer, ev), name="edl-fault",
                                 daemon=True).start()
                continue
            self._emit(s, step, trainer)
            self._fire(s, trainer)

    def _emit(self, s: FaultSpec, step: int, trainer=None) -> None:
        if self.events is not None:
            self.events.emit("fault_injected", fault=s.kind, step=step, index=self.index, point=s.point,
                             after_ms=s.after_ms or None)
        kv = getattr(trainer, "kv", None)
        if kv is not None:
            try:   # drills stop a fixed number of steps after the fault (trainer/fault_bench.py)
                kv.set("fault/fired_step", str(step))
            except Exception:  # noqa: BLE001
                pass

    def _delayed(self, s: FaultSpec, step: int, trainer, gpu_start=None) -> None:
        if gpu_start is not None:
            try:
                gpu_start.synchronize()     # the GPU starts the step now (the host enqueued it earlier)
            except Exception:  # noqa: BLE001 - fall back to the host clock
                pass
        time.sleep(s.after_ms / 1000.0)
        self._emit(s, step, trainer)
        self._fire(s, trainer)

    @staticmethod
    def _condition(s: FaultSpec, trainer) -> bool:
        """``wait=standby``: the hot standby that would replace this process is ready
        (GPU jobs: it has run its warm-up on this process's GPU)."""
        if s.wait != "standby":
            return True
        kv = getattr(trainer, "kv", None)
        if kv is None:
            return True
        from easydl_amd.utils.vram import standby_warm_on
        dev = getattr(trainer, "device", None)
        try:
            return bool(standby_warm_on(kv, dev.index if dev is not None and dev.type == "cuda" else "cpu"))
        except Exception:  # noqa: BLE001 - store unreachable: do not hold the fault back forever
            return True

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
