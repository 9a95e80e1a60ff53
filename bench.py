#!/usr/bin/env python
"""Headline benchmark: Llama-3-8B elastic-DDP training throughput (tokens/s).

Metric/config come from BASELINE.json (``tokens/sec ... Llama-3-8B elastic
DDP 1->8 GPUs``); the recovery and elasticity it drills are the reference's fault-tolerance
and elasticity claims (/root/reference/README.md:25-35).  One process per GPU; for N>1 the driver launches this file
with ``torch.distributed.run`` and every rank reads RANK / LOCAL_RANK /
WORLD_SIZE / MASTER_ADDR / MASTER_PORT from the environment; the plain form
``python bench.py --gpus N`` launches the N ranks itself (see below).

The timed loop IS the framework's elastic training loop
(:class:`easydl_amd.trainer.elastic.ElasticTrainer`): rank 0 embeds the
rendezvous master on torchrun's store, every step runs forward, backward
with the bucketed RCCL all-reduce overlapped, the store-coordinated step
commit, the global grad-norm clip and the fused AdamW update of all 8.03e9
parameters (fp32 master + moments) of the full 32-layer Llama-3-8B (random
init, synthetic tokens).  W untimed warmup steps, then exactly K steps
bracketed by barrier + synchronize; the elapsed time is the MAX over ranks;
rank 0 prints one JSON line.

Time-to-recover, the other half of the headline metric (BASELINE.json), is
measured by the plain command at any N (``python bench.py --gpus N``): this
process stays GPU-free and starts the throughput run -- one ``--child`` at
N = 1, N rank children at N > 1 (it sets RANK / LOCAL_RANK / WORLD_SIZE /
MASTER_* itself, exactly as torchrun would; never an exec of itself) -- and
then the fault drill at the SAME configuration (full Llama-3-8B, seq 8192,
2 x 4 micro-batches, in-memory snapshots every 2 steps, one hot standby):
worker N-1 is SIGKILLed 40 % into a step (counted from the GPU's start of the
step) once the standby is warm.  N = 1: the standby resumes from the dead
worker's HBM.  N > 1: the survivors shrink to N-1 and go on, the standby
rejoins, world N again, every rank ends with identical parameters.  TTR,
phases, the first recovered step's memory plan and duration, steps lost, time
to regain the pre-fault step and (N > 1) to regrow to N ranks go into
``time_to_recover_s`` / ``ttr`` of the one JSON line; a failed drill leaves
``time_to_recover_s: null`` with an ``error`` and never fails the throughput
line.  ``--ttr off`` skips the drill.  Under torchrun the launcher owns the
ranks (it tears the job down when one dies): the throughput line is the same
and ``ttr.error`` says TTR needs the plain form.
"""
from __future__ import annotations

import argparse
import json
import os
import signal
import subprocess
import sys
import time

import torch


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--model", default="llama3-8b")
    ap.add_argument("--seq", type=int, default=8192)
    # 4 micro-batches of 2 x 8k-token sequences per GPU per step (64k tokens; 512k tokens
    # per step on 8 GPUs, still below the ~1-4M-token batches Llama-3-8B pretraining uses).
    # BASELINE.json fixes the model, not the batch.  Measured on one MI355X: 2 x 1 < 2 x 2
    # (optimizer amortised, bigger GEMMs) < 2 x 4: 22.55k -> 22.82k tok/s at equal peak
    # memory (profiles/r02_bench_accum_ab.txt); on 8 GPUs the 16 GB gradient all-reduce
    # and the 38 ms AdamW are amortised over twice the tokens.
    ap.add_argument("--mbs", type=int, default=2, help="sequences per micro-batch per GPU")
    ap.add_argument("--accum", type=int, default=4, help="micro-batches per step per GPU")
    ap.add_argument("--bucket-mb", type=float, default=None)
    ap.add_argument("--grad-dtype", default=os.environ.get("EDL_GRAD_DTYPE", "bf16"), choices=["bf16", "fp32"],
                    help="gradient accumulation + all-reduce dtype (flat gradient buffers); see "
                         "docs/env_contract.md for the measured trade-off")
    ap.add_argument("--layers", type=int, default=None,
                    help="override layer count (debug only; invalid for the metric)")
    ap.add_argument("--out", default=None)
    ap.add_argument("--ckpt-interval", type=int, default=0,
                    help="in-memory sharded snapshot every K steps (async D2H, overlapped)")
    ap.add_argument("--fault-inject", action="store_true", help="measure time-to-recover instead (local operator)")
    ap.add_argument("--scale-up", default=None, metavar="START:END",
                    help="measure an elastic scale-up mid-run instead (BASELINE config 2, ResNet-50)")
    ap.add_argument("--share-gpu", action="store_true",
                    help="--fault-inject: all --gpus workers on GPU 0 over the xGMI engine (shrink on one GPU)")
    ap.add_argument("--fault-step", type=int, default=None, help="--fault-inject: step at which the worker dies")
    ap.add_argument("--standby", type=int, default=1,
                    help="--fault-inject: warm spare workers kept by the operator (0 = cold respawn)")
    ap.add_argument("--comm", default=None, choices=["pg", "xgmi", "auto", "xgmi-only", "auto-gloo"],
                    help="gradient all-reduce data plane (default $EDL_COMM or auto = RCCL + the hand-written xGMI "
                         "engine, per-size policy probed once per (group, world) and cached; pg = ProcessGroupNCCL "
                         "(RCCL) only; xgmi = engine for every all-reduce; "
                         "auto-gloo = auto with gloo standing in for RCCL (ranks sharing one GPU: tests, drills)")
    ap.add_argument("--sp", action="store_true", help="Megatron sequence parallelism inside the TP group")
    ap.add_argument("--tp", type=int, default=1,
                    help="tensor-parallel degree inside each DP replica (BASELINE config 5: --model llama3-70b --tp 8)")
    ap.add_argument("--fault-mode", default="midstep", choices=["midstep", "in_update", "step_start"],
                    help="--fault-inject: where the kill lands (trainer/fault_bench.py)")
    ap.add_argument("--ttr", default="auto", choices=["auto", "off"],
                    help="N=1 on a GPU host: also run the time-to-recover drill at this config (auto)")
    ap.add_argument("--ttr-timeout", type=float, default=float(os.environ.get("EDL_TTR_TIMEOUT", 330)),
                    help="seconds the time-to-recover drill may take before it is abandoned")
    ap.add_argument("--moments", default="auto", choices=["auto", "fp32", "bf16"],
                    help="AdamW moment dtype; auto = bf16 only when fp32 moments would not fit two full in-memory "
                         "snapshot slots in this rank's host DRAM (config 5), else fp32")
    ap.add_argument("--child", action="store_true", help=argparse.SUPPRESS)
    return ap.parse_args()


def _json_line(text: str) -> dict | None:
    for ln in reversed((text or "").splitlines()):
        ln = ln.strip()
        if ln.startswith("{"):
            try:
                return json.loads(ln)
            except ValueError:
                continue
    return None


def _run_child(argv: list[str], timeout_s: float, env: dict | None = None) -> tuple[int | None, str]:
    """Run ``argv`` in its own process group (stderr passes through); on timeout the whole
    group (operator, workers, standbys of a drill) is killed.  Returns (rc or None, stdout)."""
    p = subprocess.Popen(argv, stdout=subprocess.PIPE, text=True, env=env, start_new_session=True)
    try:
        out, _ = p.communicate(timeout=timeout_s)
        return p.returncode, out
    except subprocess.TimeoutExpired:
        try:
            os.killpg(p.pid, signal.SIGKILL)
        except OSError:
            pass
        out, _ = p.communicate()
        return None, out


def _gpu_host() -> bool:
    """GPUs on this host, found without initialising HIP in this process (KFD sysfs)."""
    try:
        from easydl_amd.brain.collectors import kfd_gpus
        return bool(kfd_gpus())
    except Exception:  # noqa: BLE001
        return False


def _free_port() -> int:
    import socket
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        return sk.getsockname()[1]


def _launch_ranks(args, n: int, timeout_s: float) -> tuple[int | None, str]:
    """N > 1 from the plain command: this GPU-free process starts N rank processes of this file
    itself, with the environment torchrun would give them (RANK / LOCAL_RANK / WORLD_SIZE /
    LOCAL_WORLD_SIZE / MASTER_ADDR / MASTER_PORT; rank 0 hosts the job store).  Each is a child
    process in its own session -- never an exec of this one.  A rank that fails ends the others.
    Returns (rc or None on timeout, rank 0's stdout)."""
    me = os.path.abspath(__file__)
    port = _free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   GROUP_RANK="0", ROLE_RANK=str(r), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        env.pop("TORCHELASTIC_USE_AGENT_STORE", None)
        procs.append(subprocess.Popen([sys.executable, me, *sys.argv[1:], "--child"], env=env, text=True,
                                      stdout=subprocess.PIPE if r == 0 else subprocess.DEVNULL,
                                      start_new_session=True))
    out = []
    reader = __import__("threading").Thread(target=lambda: out.append(procs[0].stdout.read()), daemon=True)
    reader.start()
    t_end = time.monotonic() + timeout_s
    rc = 0
    live = set(range(n))
    while live and time.monotonic() < t_end:
        for r in sorted(live):
            c = procs[r].poll()
            if c is None:
                continue
            live.discard(r)
            if c != 0:
                rc = c
                print(f"[bench] rank {r} exited with {c}: stopping the other ranks", file=sys.stderr)
                live.clear()
                break
        time.sleep(0.05)
    if live or rc:
        rc = None if live else rc
        for p in procs:
            if p.poll() is None:
                try:
                    os.killpg(p.pid, signal.SIGKILL)
                except OSError:
                    pass
    for p in procs:
        p.wait()
    reader.join(10)
    return rc, "".join(out)


def _drill(args, res: dict, n: int) -> dict:
    """The time-to-recover drill at the headline configuration, after the throughput run.
    N = 1: the only worker is SIGKILLed 40 % into a step once the hot standby is warm; the
    standby resumes from the dead worker's HBM.  N > 1: worker N-1 is SIGKILLed the same way;
    the N-1 survivors abort, shrink and go on; the hot standby takes the dead worker's place and
    rejoins (world N again); every final rank must hold the same parameters."""
    me = os.path.abspath(__file__)
    ttr = {"mode": "midstep", "hot_standby": 1, "ckpt_interval": 2, "workers": n}
    t0 = time.perf_counter()
    try:
        from easydl_amd.ckpt.manager import unlink_job_segments
        unlink_job_segments("bench")
        env = dict(os.environ, EDL_FAULT_STEP_MS=str(res["ms_per_step"]))
        if n > 1:
            env.setdefault("EDL_BENCH_UNTIL_REGROWN", "1")    # end once the replacement is back in
        for k in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "LOCAL_WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT"):
            env.pop(k, None)
        drill = [sys.executable, me, "--fault-inject", "--gpus", str(n), "--model", args.model, "--seq",
                 str(args.seq), "--mbs", str(args.mbs), "--accum", str(args.accum), "--ckpt-interval", "2",
                 "--standby", "1", "--fault-mode", "midstep", "--fault-step", "4", "--steps", "0", "--warmup", "0"]
        if args.layers:
            drill += ["--layers", str(args.layers)]
        timeout = args.ttr_timeout if n == 1 else max(args.ttr_timeout, 480.0)
        drc, dout = _run_child(drill, timeout_s=timeout, env=env)
        d = _json_line(dout)
        ttr["drill_wall_s"] = round(time.perf_counter() - t0, 1)
        if d is None or d.get("value") is None:
            ttr["error"] = ("drill timed out" if drc is None else f"drill rc={drc}") + \
                ("" if d is None else f", no recovery in the timeline: {json.dumps(d.get('breakdown'))[:300]}")
            return ttr
        res["time_to_recover_s"] = d["value"]
        b = d.get("breakdown") or {}
        finals = d.get("final_states") or []
        ttr.update({
            "time_to_regain_s": d.get("time_to_regain_s"), "steps_lost": d.get("steps_lost"),
            "time_to_regrow_s": d.get("time_to_regrow_s"), "worlds_seen": d.get("worlds_seen"),
            "restored_from": d.get("restored_from"), "resumed_mid_step": d.get("resumed_mid_step"),
            "grad_shadow": d.get("grad_shadow"),
            "fault_step": (d.get("fault") or {}).get("step"),
            "fault_spec": (d.get("fault") or {}).get("spec"),
            "replacement_from_standby": d.get("replacement_from_standby"),
            "step_s_before_fault": d.get("step_s_before_fault"),
            "step_s_before_fault_clock": d.get("step_s_before_fault_clock"),
            "gpu_steps_before_fault": d.get("gpu_steps_before_fault"),
            "step_s_steady": round(res["ms_per_step"] / 1e3, 4),    # the throughput run's step
            "standby_slab_gb": d.get("standby_slab_gb"),
            "first_step": d.get("first_step"),
            "phases": {k: b.get(k) for k in ("detect_s", "abort_s", "epoch_formed_s", "replacement_spawn_s",
                                             "replacement_joined_s", "comm_ready_s", "state_synced_s",
                                             "first_step_s")},
            "final_ranks": len(finals),
            "final_states_equal": len({json.dumps(f.get("crc")) for f in finals}) == 1 if finals else None,
            "final_worlds": sorted({f.get("world") for f in finals if f.get("world")}),
            "timeline": d.get("timeline"),
            "config": d.get("config"), "model": d.get("model"), "operator_rc": d.get("operator_rc")})
    except Exception as e:  # noqa: BLE001 - the drill never fails the throughput line
        ttr["error"] = f"{type(e).__name__}: {e}"[:300]
    return ttr


def parent(args) -> int:
    """The plain command at any N: the throughput run (one child at N = 1, N rank children at
    N > 1), then the time-to-recover drill child at the same configuration; one JSON line."""
    n = max(1, args.gpus)
    if n > 1 and _gpu_host():
        from easydl_amd.brain.collectors import kfd_gpus
        have = len(kfd_gpus())
        if have < n:
            print(f"[bench] --gpus {n} but this host has {have} GPU(s)", file=sys.stderr)
            return 2
    me = os.path.abspath(__file__)
    if n == 1:
        rc, out = _run_child([sys.executable, me, *sys.argv[1:], "--child"], timeout_s=3600)
    else:
        rc, out = _launch_ranks(args, n, timeout_s=3600)
    res = _json_line(out)
    if rc != 0 or res is None:
        sys.stdout.write(out)
        print(f"[bench] throughput run failed (rc={rc})", file=sys.stderr)
        return rc if rc else 1
    if n > 1:
        res["launch"] = f"bench.py parent: {n} rank processes (RANK/LOCAL_RANK/WORLD_SIZE set by it)"
    if args.ttr == "off":
        res["ttr"] = {"skipped": "--ttr off"}
    elif args.tp > 1:
        res["ttr"] = {"error": "the time-to-recover drill runs the data-parallel headline only (--tp 1)"}
    else:
        res["ttr"] = _drill(args, res, n)
    print(json.dumps(res), flush=True)
    if args.out:
        with open(args.out, "w") as f:
            f.write(json.dumps(res) + "\n")
    return 0


def main():
    args = parse()
    plain = not (args.child or args.fault_inject or args.scale_up or args.share_gpu)
    if plain and "WORLD_SIZE" not in os.environ and args.gpus > 1:
        return parent(args)          # N ranks launched from here, then the N-rank drill
    if (plain and args.ttr == "auto" and os.environ.get("WORLD_SIZE", "1") == "1" and args.tp == 1
            and _gpu_host()):
        return parent(args)
    if args.fault_inject:
        from easydl_amd.trainer import fault_bench
        return fault_bench.main(args)
    if args.scale_up:
        from easydl_amd.trainer import scale_bench
        start, end = args.scale_up.split(":")
        return scale_bench.main(["--start", start, "--end", end, "--steps", str(args.warmup + args.steps)]
                                + (["--share-gpu"] if args.share_gpu else []))
    rank = int(os.environ.get("RANK", 0))
    world = int(os.environ.get("WORLD_SIZE", 1))
    local = int(os.environ.get("LOCAL_RANK", 0))
    if world != args.gpus and rank == 0:
        print(f"[bench] note: --gpus {args.gpus} but WORLD_SIZE={world}; using WORLD_SIZE", file=sys.stderr)
    use_cuda = torch.cuda.is_available()
    dev = torch.device("cuda", 0 if args.share_gpu else local) if use_cuda else torch.device("cpu")
    if args.share_gpu and use_cuda:
        # every rank on GPU 0, the xGMI engine as the only data plane (test / fault drills
        # on a one-GPU box; not the headline configuration); --comm auto-gloo overrides
        os.environ["EDL_COMM"] = "xgmi-only"
        os.environ.setdefault("EDL_XGMI_MAX_BLOCKS", "16")   # co-residency of all ranks' grids
    os.environ.setdefault("EDL_JOB", "bench")
    if args.comm:
        os.environ["EDL_COMM"] = args.comm
    if args.sp:
        os.environ["EDL_SP"] = "1"
    os.environ.setdefault("EDL_RUN_DIR", os.path.join("gpurun_out", "bench_run") if use_cuda else "/tmp/edl_bench")

    from easydl_amd.models.llama import Llama, get_config
    from easydl_amd.trainer.data import SyntheticTokens
    from easydl_amd.trainer.elastic import ElasticTrainer

    overrides = {"n_layers": args.layers} if args.layers else {}
    cfg = get_config(args.model, **overrides)
    dtype = torch.bfloat16 if use_cuda else torch.float32
    S, B = args.seq, args.mbs
    tp = args.tp
    if world % tp:
        raise SystemExit(f"WORLD_SIZE={world} is not a multiple of --tp {tp}")
    dp = world // tp
    gb = dp * B * args.accum
    ckpt = None
    if args.ckpt_interval > 0:
        from easydl_amd.ckpt.manager import CheckpointManager, unlink_job_segments
        unlink_job_segments("bench")
        ckpt = CheckpointManager("bench", interval=args.ckpt_interval)
    if tp > 1:
        from easydl_amd.parallel.tp import LlamaTP
        model_fn = lambda d, g: LlamaTP(cfg, g, device=d, dtype=dtype)  # noqa: E731
    else:
        model_fn = lambda d: Llama(cfg, device=d, dtype=dtype)  # noqa: E731
    tr = ElasticTrainer(model_fn, lr=3e-4, betas=(0.9, 0.95), weight_decay=0.1,
                        max_grad_norm=1.0, global_batch=gb, micro_batch=B, device=dev, bucket_mb=args.bucket_mb,
                        checkpoint=ckpt, tp=tp, moment_dtype=args.moments,
                        grad_dtype=torch.float32 if (args.grad_dtype == "fp32" or not use_cuda) else torch.bfloat16)
    marks = {}

    def sync_barrier(t):
        if use_cuda:
            torch.cuda.synchronize(dev)
        t.comm.barrier()

    def on_step(t, loss):
        if t.step == args.warmup:
            sync_barrier(t)
            marks["t0"] = time.perf_counter()
            marks["warm_end"] = time.perf_counter()
        if t.step == args.warmup + args.steps:
            sync_barrier(t)
            marks["t1"] = time.perf_counter()

    t_start = time.perf_counter()
    tr.fit(lambda m, b: m(*b), SyntheticTokens(cfg.vocab_size, S), num_steps=args.warmup + args.steps,
           on_step=on_step)
    comm = tr.comm
    el = marks["t1"] - marks["t0"]
    if comm.world_size > 1:
        import torch.distributed as dist
        el = float(comm.ctrl_all_reduce([el], op=dist.ReduceOp.MAX)[0])
    tokens = (comm.world_size // tp) * B * S * args.accum * args.steps
    tps = tokens / el
    fpt = cfg.flops_per_token(S)
    tflops_gpu = tps / (1 if (args.share_gpu and use_cuda) else comm.world_size) * fpt / 1e12
    dp_world = comm.world_size // tp
    if dp_world > 1:
        metric = "tokens/sec, Llama-3-8B elastic DDP (full train step: fwd+bwd+bucketed all-reduce+commit+AdamW)"
    else:
        # one data-parallel rank: the gradient all-reduce is the identity (LocalCommunicator)
        # and no rendezvous commit runs; the step is fwd+bwd+clip+AdamW
        metric = ("tokens/sec, Llama-3-8B elastic DDP "
                  "(full train step at N=1: fwd+bwd+clip+AdamW; all-reduce is identity)")
    if tp > 1:
        metric = f"tokens/sec, {args.model} elastic DP x TP={tp} (full train step)"
    res = {
        "metric": metric,
        "value": round(tps, 2),
        "unit": "tokens/s",
        "n_gpus": 1 if (args.share_gpu and use_cuda) else comm.world_size,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(el / args.steps * 1e3, 3),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "bf16" if use_cuda else "fp32",
        "data": "synthetic (random token ids), random-init weights",
        "config": {
            "model": args.model if not args.layers else f"{args.model}-L{args.layers}",
            "global_batch": gb,
            "seq_len": S,
            "parallelism": f"dp{comm.world_size // tp}" + (f"tp{tp}" if tp > 1 else "") + ("sp" if args.sp else ""),
            "micro_batch": B,
            "grad_accum": args.accum,
            "optimizer": f"AdamW fp32 master, {str(getattr(tr.opt, 'moment_dtype', 'fp32')).replace('torch.', '')}"
                         " moments, clip 1.0",
            "grad_dtype": str(tr.flat.grad_dtype).replace("torch.", "") if tr.flat is not None else args.grad_dtype,
            "bucket_mb": tr.ddp.bucket_mb,
            "comm": getattr(getattr(comm, "dp", comm), "backend", "local"),
            "gemm_tuning": getattr(tr, "gemm_tuning", "off"),
        },
        "ranks": comm.world_size,
        "shared_gpu": bool(args.share_gpu and use_cuda),   # functional drill, not a throughput figure
        "allreduce_probe": getattr(getattr(comm, "dp", comm), "xgmi_probe", None),
        "tflops_per_gpu": round(tflops_gpu, 1),
        "mfu_vs_2.5PF": round(tflops_gpu / 2500.0, 4),
        "loss": round(float(tr.last_loss), 4) if tr.last_loss is not None else None,
        "peak_mem_gb": round(torch.cuda.max_memory_allocated(dev) / 2**30, 1) if use_cuda else 0.0,
        "setup_and_warmup_s": round(marks["t0"] - t_start, 2),
        # N=1 on a GPU host: filled in by the parent from the drill; otherwise see --fault-inject
        "time_to_recover_s": None,
        "ckpt": None if ckpt is None else {
            "interval": args.ckpt_interval, "snapshots": ckpt.stats["snapshots"],
            "bytes_per_snapshot": ckpt.stats["d2h_bytes"] // max(1, ckpt.stats["snapshots"]),
            "pinned": ckpt.pin, "staged_last": ckpt.stats.get("staged_last"),
            "mode": ckpt.mode, "host_budget_gb": ckpt.stats.get("host_budget_gb")},
    }
    if not args.child and comm.world_size > 1:
        # launched by torchrun: the launcher owns the ranks and tears the job down when one dies
        res["ttr"] = {"error": "time-to-recover needs the plain form `python bench.py --gpus N` (its parent "
                               "launches the N ranks, then the N-rank kill -> shrink -> rejoin drill); under "
                               "torchrun a killed rank ends the whole launch"}
    if comm.rank == 0:
        line = json.dumps(res)
        print(line, flush=True)
        if args.out:
            with open(args.out, "w") as f:
                f.write(line + "\n")
    tr.close()
    if ckpt is not None:
        ckpt.close()
        from easydl_amd.ckpt.manager import unlink_job_segments
        unlink_job_segments("bench")


if __name__ == "__main__":
    sys.exit(main())
