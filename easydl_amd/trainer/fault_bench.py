"""Time-to-recover benchmark (``bench.py --fault-inject``; BASELINE.json metric
"time-to-recover ... w/ fault inject", config 3 "kill-1-worker fault inject +
in-mem ckpt restore").

Runs a real job through the local ElasticOperator on this node's GPUs (or CPU
processes when no GPU is visible):

* N workers train the model with in-memory sharded snapshots every
  ``--ckpt-interval`` steps;
* worker ``N-1`` SIGKILLs itself at step ``--fault-step`` (EDL_FAULT);
* N > 1: the supervisor's pidfd exit event reaches the master in
  microseconds, the epoch is aborted, survivors abort RCCL, rebuild an (N-1)
  world and continue without restarting; the operator's replacement later
  rejoins (scale-up with state broadcast);
* N = 1: there is no survivor: the replacement process restores the newest
  committed snapshot from /dev/shm and continues.

TTR = wall time from the ``fault_injected`` event to the first committed step
after it; the breakdown (detect / abort / new epoch / comm ready / state sync
/ first step) comes from the merged event timeline.  ``time_to_regain_s`` is
the time until the job holds its pre-fault committed step count again.  Prints
one JSON line.

Where the kill lands (``--fault-mode``, utils/fault.py):

* ``midstep`` (default): 40 % into a step (``after_ms``), once the hot standby
  has warmed up -- a failure at an arbitrary moment, with that step's GPU work
  in flight;
* ``in_update``: inside an optimizer update (after its ``begin`` step mark), so
  the dead worker's HBM is torn and the state comes back from /dev/shm;
* ``step_start``: at the host's start of step ``--fault-step`` (round-1..4 form).

After the fault every process trains ``EDL_BENCH_AFTER`` (default 3) more steps
past the fault step and the job ends.
"""
from __future__ import annotations

import json
import os
import shutil
import sys
import tempfile

from easydl_amd.utils.events import read_events, ttr_breakdown


def _gpus() -> list[int]:
    from easydl_amd.brain.collectors import kfd_gpus
    return [g.index for g in kfd_gpus()]


def main(args) -> int:
    from easydl_amd.api.spec import ElasticJob, JobResource, Resource, RoleResource
    from easydl_amd.ckpt.manager import unlink_job_segments
    from easydl_amd.operator.reconciler import ElasticOperator, OperatorConfig

    gpus = _gpus()
    share = bool(getattr(args, "share_gpu", False)) and bool(gpus)
    if share:
        # N workers on ONE GPU, the xGMI engine as the only data plane (RCCL refuses two
        # ranks on one device): worker death -> shrink measured on a single MI355X
        n = max(1, args.gpus)
        gpus = [gpus[0]] * n
    else:
        n = max(1, min(args.gpus, len(gpus))) if gpus else max(1, args.gpus)
    run_dir = tempfile.mkdtemp(prefix="edl-ttr-", dir=os.environ.get("EDL_TTR_DIR", None))
    job_name = "ttr"
    unlink_job_segments(job_name)
    steps = args.warmup + args.steps
    fault_step = getattr(args, "fault_step", None) or max(2, args.warmup + 1)
    mode = getattr(args, "fault_mode", None) or "step_start"
    standby = getattr(args, "standby", 0)
    spec = f"kill@step={fault_step},index={n - 1}"
    if mode == "midstep":
        # 40 % into the step at its steady length (EDL_FAULT_STEP_MS: the caller's measured
        # step time; else a guess from the model), so the step's GPU work is in flight
        spec += f",after_ms={int(float(os.environ.get('EDL_FAULT_STEP_MS', 1000)) * 0.4)}"
    elif mode == "in_update":
        spec += ",point=in_update"
    if standby and mode != "step_start":
        spec += ",wait=standby"   # a real failure finds the spare parked and warmed up
    spec = os.environ.get("EDL_BENCH_FAULT_SPEC") or spec   # e.g. a second kill of the replacement (gen=1)
    env = {
        "EDL_BENCH_MODEL": args.model, "EDL_BENCH_SEQ": str(args.seq), "EDL_BENCH_MBS": str(args.mbs),
        "EDL_BENCH_ACCUM": str(args.accum),
        # step_start keeps the fixed step count; the other modes end a few steps after the fault
        "EDL_BENCH_STEPS": str(steps if mode == "step_start" else
                               fault_step + int(os.environ.get("EDL_BENCH_CAP", 60))),
        "EDL_BENCH_AFTER": os.environ.get("EDL_BENCH_AFTER", "3" if mode != "step_start" else "0"),
        "EDL_BENCH_CKPT": str(getattr(args, "ckpt_interval", 0) or 2),
        "EDL_FAULT": spec,
        "EDL_PLANNED_WORKERS": str(n),
    }
    if args.layers:
        env["EDL_BENCH_LAYERS"] = str(args.layers)
    if share:
        # xgmi-only by default; --comm auto-gloo runs the DEFAULT auto plane (engine probe,
        # policy cache, deferral) with gloo on GPU tensors standing in for RCCL
        env["EDL_COMM"] = getattr(args, "comm", None) or "xgmi-only"
        env["EDL_XGMI_MAX_BLOCKS"] = "16"   # all ranks' grids must be co-resident on the one GPU
    elif getattr(args, "comm", None):
        env["EDL_COMM"] = args.comm
    job = ElasticJob(name=job_name, command="python -m easydl_amd.trainer.fault_bench --worker",
                     env=env, min_workers=1, max_workers=n)
    for k in ("EDL_BENCH_UNTIL_REGROWN",):
        if k in os.environ:
            env[k] = os.environ[k]
    jr = JobResource(f"{job_name}-resource", job_name,
                     {"worker": RoleResource(n, Resource(gpu=1 if gpus else 0, cpu=4 if gpus else 1))})
    cfg = OperatorConfig(gpus=gpus[:n], cpus=[], leave_grace_s=120.0, standby=getattr(args, "standby", 0))
    op = ElasticOperator(job, run_dir, cfg=cfg, job_resource=jr)
    rc = op.run(timeout_s=1000)
    ev = read_events(run_dir)
    ttr = ttr_breakdown(ev)
    worlds = [e.get("world") for e in ev if e["kind"] == "step_done"]
    restored = [e for e in ev if e["kind"] == "restored"]
    fault = next((e for e in ev if e["kind"] == "fault_injected"), None)
    done_ts = [e["ts"] for e in ev if e["kind"] == "step_done" and (fault is None or e["ts"] < fault["ts"])]
    gaps = sorted(b - a for a, b in zip(done_ts, done_ts[1:]))[-8:]   # the last steps before the fault
    steady = sorted(b - a for a, b in zip(done_ts[2:], done_ts[3:]))     # every step before it, first 3 out
    # GPU step durations (start of step k's forward -> end of its update, HIP events, ElasticTrainer
    # _mark_gpu_step_start/_end): at world 1 the host enqueues ahead of the GPU, so host gaps are not steps
    timed = {int(e["gpu_step"]): (e["gpu_s"], bool(e.get("gpu_after_snapshot"))) for e in ev
             if e["kind"] == "step_done" and e.get("gpu_s") is not None and (fault is None or e["ts"] < fault["ts"])
             and int(e.get("gpu_step", 0)) >= 2}
    # the median excludes steps whose update waited for a snapshot's device-to-host copy (the first
    # snapshots also create and pin their segments: seconds)
    gpu = sorted(v for v, snap in timed.values() if not snap) or sorted(v for v, _ in timed.values())
    out = {
        "metric": "time-to-recover after SIGKILL of one worker (Llama elastic DDP, local operator)",
        "value": None if not ttr else ttr["ttr_s"], "unit": "s", "higher_is_better": False,
        "n_gpus": (1 if share else n) if gpus else 0,
        "model": (args.model if not args.layers else f"{args.model}-L{args.layers}") if gpus else "llama-tiny (CPU)",
        "config": {"seq_len": args.seq if gpus else 64, "micro_batch": args.mbs, "grad_accum": args.accum,
                   "ckpt_interval": int(env["EDL_BENCH_CKPT"])},
        "fault": {"mode": mode, "spec": spec, "step": fault.get("step") if fault else None},
        "breakdown": ttr, "operator_rc": rc, "hot_standby": standby,
        "time_to_regain_s": ttr.get("time_to_regain_s") if ttr else None,
        "steps_lost": ttr.get("steps_lost") if ttr else None,
        "step_s_before_fault": (round(gpu[len(gpu) // 2], 4) if gpu else
                                round(gaps[len(gaps) // 2], 4) if gaps else None),
        "step_s_before_fault_clock": "gpu" if gpu else "host",
        # every GPU-timed step before the fault
        "gpu_steps_before_fault": {str(k): {"s": round(v, 4), "after_snapshot": snap}
                                   for k, (v, snap) in sorted(timed.items())},
        "first_step": _first_step(ev, fault, ttr),
        "time_to_regrow_s": _regrow(ev, fault, n),
        "step_s_median": round(steady[len(steady) // 2], 5) if steady else None,
        "shared_gpu": share, "comm": env.get("EDL_COMM", "pg"), "workers": n,
        "replacement_from_standby": any(e["kind"] == "spawn" and e.get("standby") for e in ev),
        "restored_from": restored[0].get("source") if restored else None,
        "hbm_resume_refused": any(e["kind"] == "hbm_resume_refused" for e in ev),
        "resumed_mid_step": next(({k: e.get(k) for k in ("step", "micro_batches_done", "of")}
                                  for e in ev if e["kind"] == "resumed_mid_step"), None),
        "grad_shadow": next(({k: e.get(k) for k in ("on", "where", "gb", "free_gb", "replacement_need_gb")}
                             for e in ev if e["kind"] == "grad_shadow"), None),
        "final_states": [{k: e.get(k) for k in ("proc", "step", "world", "rank", "crc")}
                         for e in ev if e["kind"] == "final_state"],
        "worlds_seen": sorted({w for w in worlds if w}), "run_dir": run_dir,
        "timeline": _timeline(ev, fault, ttr),
        "standby_slab_gb": _slab_gb(run_dir),
    }
    print(json.dumps(out), flush=True)
    unlink_job_segments(job_name)
    if os.environ.get("EDL_TTR_KEEP") != "1":
        shutil.rmtree(run_dir, ignore_errors=True)
    return 0 if rc == 0 and ttr else 1


def _slab_gb(run_dir: str) -> float | None:
    """HBM the parked standby had reserved for the replacement's first step (its log line)."""
    import glob
    import re
    for f in glob.glob(os.path.join(run_dir, "logs", "*standby*.log")):
        with open(f, errors="replace") as fh:
            m = re.findall(r"slab ([0-9.]+) GB", fh.read())
        if m:
            return float(m[-1])
    return None


def _rel(e, fault):
    return None if e is None or fault is None else round(e["ts"] - fault["ts"], 4)


def _first_step(ev: list[dict], fault, ttr) -> dict | None:
    """The first committed step after the fault: its own duration, and the memory plan it ran
    under (a takeover short of HBM: split / recomputed layers, ElasticTrainer _memory_plan) with
    when the memory came back -- the evidence of where a time-to-recover went."""
    if fault is None or not ttr or ttr.get("first_step_s") is None:
        return None
    t_done = fault["ts"] + ttr["first_step_s"]
    after = [e for e in ev if e["ts"] >= fault["ts"]]
    done = next((e for e in after if e["kind"] == "step_done" and abs(e["ts"] - t_done) < 1e-3), None)
    plan = next((e for e in after if e["kind"] == "memory_limited_steps"), None)
    restored = next((e for e in after if e["kind"] == "memory_restored"), None)
    pieces = next((e for e in after if e["kind"] == "limited_step_pieces"), None)
    return {
        "s": done.get("dt") if done else None, "proc": done.get("proc") if done else None,
        "pieces": None if pieces is None else {"gpu_s": pieces.get("gpu_s"), "host_s": pieces.get("host_s"),
                                               "each": pieces.get("pieces")},
        "world": done.get("world") if done else None,
        "memory_plan": None if plan is None else {k: plan.get(k) for k in (
            "split", "recompute_layers", "layers", "need_gb", "avail_gb", "margin")},
        "memory_replans": sum(1 for e in after if e["kind"] == "memory_replanned" and e["ts"] <= t_done),
        "memory_restored_s": _rel(restored, fault),
        "memory_restored_at": None if restored is None else {"step": restored.get("step"), "mb": restored.get("mb"),
                                                             "avail_gb": restored.get("avail_gb")},
    }


def _regrow(ev: list[dict], fault, n: int) -> float | None:
    """N > 1: fault -> the first committed step at the full world size again (the replacement rejoined)."""
    if fault is None or n <= 1:
        return None
    formed = next((x for x in ev if x["kind"] == "epoch_formed" and x["ts"] > fault["ts"] and x.get("world") == n),
                  None)
    if formed is None:
        return None
    done = next((d for d in ev if d["kind"] == "step_done" and d["ts"] > formed["ts"] and d.get("world") == n), None)
    return _rel(done, fault)


_TIMELINE_KINDS = ("fault_injected", "node_dead", "epoch_abort", "epoch_formed", "spawn", "exit_early", "joined",
                   "restored", "comm_ready", "state_synced", "state_broadcast", "memory_limited_steps",
                   "memory_replanned", "memory_restored", "step_done", "hbm_resume_refused", "rehomed")


def _timeline(ev: list[dict], fault, ttr, limit: int = 48) -> list[dict]:
    """Compact event timeline from the fault to one second past the first recovered step (the
    drill's run directory is temporary: this is what stays in the JSON)."""
    if fault is None:
        return []
    end = fault["ts"] + ((ttr or {}).get("first_step_s") or 30.0) + 1.0
    out, seen = [], {}
    for e in ev:
        if e["ts"] < fault["ts"] or e["ts"] > end or e["kind"] not in _TIMELINE_KINDS:
            continue
        key = (e["kind"], e.get("epoch"), e.get("world"), e.get("step"))
        if key in seen:     # N ranks doing the same thing: the first one, with a count
            seen[key]["ranks"] = seen[key].get("ranks", 1) + 1
            continue
        rec = seen[key] = {"t": _rel(e, fault), "proc": e.get("proc"), "kind": e["kind"]}
        for k in ("step", "epoch", "world", "dt", "split", "recompute_layers", "need_gb", "avail_gb", "source",
                  "mb", "gpu_free_gb"):
            if e.get(k) is not None:
                rec[k] = e[k]
        out.append(rec)
    return out[:limit]


def worker() -> None:
    """One training process of the TTR job (spawned by the operator)."""
    import torch

    from easydl_amd.ckpt.manager import CheckpointManager
    from easydl_amd.models.llama import Llama, get_config
    from easydl_amd.trainer.data import SyntheticTokens
    from easydl_amd.trainer.elastic import ElasticTrainer

    e = os.environ
    over = {"n_layers": int(e["EDL_BENCH_LAYERS"])} if "EDL_BENCH_LAYERS" in e else {}
    cfg = get_config(e.get("EDL_BENCH_MODEL", "llama3-8b"), **over)
    cuda = torch.cuda.is_available()
    if not cuda:
        cfg = get_config("llama-tiny")
    seq = int(e.get("EDL_BENCH_SEQ", 8192)) if cuda else 64
    mbs, accum = int(e.get("EDL_BENCH_MBS", 1)), int(e.get("EDL_BENCH_ACCUM", 1))
    ckpt = CheckpointManager(e.get("EDL_JOB", "ttr"), interval=int(e.get("EDL_BENCH_CKPT", 2)))
    tr = ElasticTrainer(lambda d: Llama(cfg, device=d, dtype=torch.bfloat16 if cuda else torch.float32),
                        global_batch=None, micro_batch=mbs, checkpoint=ckpt)
    # global batch: the planned world x mbs x accum, fixed across resizes (accumulation absorbs it)
    tr.global_batch = mbs * accum * max(1, int(e.get("EDL_PLANNED_WORKERS", 1)))
    after = int(e.get("EDL_BENCH_AFTER", 0))

    planned = max(1, int(e.get("EDL_PLANNED_WORKERS", 1)))
    regrow = e.get("EDL_BENCH_UNTIL_REGROWN", "0") == "1"

    def on_step(t, _loss):
        # every rank reads the same store key at the same committed step: they stop together
        # (with EDL_BENCH_UNTIL_REGROWN=1 only once the replacement has rejoined: world size is
        # the same on every rank of an epoch)
        if after > 0 and getattr(t, "kv", None) is not None:
            fired = t.kv.get_str("fault/fired_step")
            if fired is not None and t.step >= int(fired) + after and (
                    not regrow or t.comm.world_size >= planned):
                t.request_stop()

    tr.fit(lambda m, b: m(*b), SyntheticTokens(cfg.vocab_size, seq), num_steps=int(e.get("EDL_BENCH_STEPS", 10)),
           on_step=on_step)
    # final state digest per rank: a drill checks every rank ended with the same parameters
    import zlib
    if tr.device.type == "cuda":
        from easydl_amd.ckpt.manager import checksum_tensor
        digest = [int(checksum_tensor(g.data).item()) for g in tr.flat.groups]
    else:
        digest = [zlib.crc32(g.data.detach().float().numpy().tobytes()) for g in tr.flat.groups]
    tr.events.emit("final_state", step=tr.step, world=tr.comm.world_size if tr.comm is not None else None,
                   rank=tr.comm.rank if tr.comm is not None else None, crc=digest)
    tr.close()
    ckpt.close()


if __name__ == "__main__":
    if "--worker" in sys.argv:
        worker()
