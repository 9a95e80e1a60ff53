"""``edl`` command line.

    python -m easydl_amd.cli submit job.yaml [--gpus 0,1,...] [--run-dir DIR]
        run the local ElasticOperator in the foreground: it creates the job
        master first; the master gets a plan from the Brain (or uses the
        JobResource in the same YAML) and the operator reconciles processes.
    python -m easydl_amd.cli apply jobresource.yaml --job NAME --port P
        update the JobResource of a running job (scale / replace).
    python -m easydl_amd.cli status --job NAME --port P
    python -m easydl_amd.cli scale --job NAME --port P --workers N
    python -m easydl_amd.cli kill  --job NAME --port P --node NODE   (fault injection)
    python -m easydl_amd.cli brain [--port 8808]
"""
from __future__ import annotations

import argparse
import json
import logging
import os
import sys


def _kv(a):
    from easydl_amd.master.store import KV, make_tcp_store
    return KV(make_tcp_store(a.host, a.port, False, timeout_s=10), f"edl/{a.job}")


def cmd_submit(a):
    from easydl_amd.api.spec import load_specs
    from easydl_amd.operator.reconciler import ElasticOperator, OperatorConfig
    job, jr = load_specs(a.spec)
    if job is None:
        raise SystemExit("spec has no ElasticJob")
    gpus = [int(g) for g in a.gpus.split(",")] if a.gpus else _detect_gpus()
    cfg = OperatorConfig(gpus=gpus, cpus=list(range(os.cpu_count() or 1)), master_port=a.master_port,
                         standby=a.standby)
    op = ElasticOperator(job, a.run_dir or os.path.join("runs", job.name), cfg=cfg, job_resource=jr)
    print(json.dumps({"job": job.name, "master_port": op.master_port, "run_dir": op.run_dir}), flush=True)
    return op.run(timeout_s=a.timeout)


def _detect_gpus():
    from easydl_amd.brain.collectors import kfd_gpus
    return [g.index for g in kfd_gpus()]


def cmd_apply(a):
    from easydl_amd.api.spec import load_specs
    _, jr = load_specs(a.spec)
    kv = _kv(a)
    cur = kv.get("jobresource")
    jr.version = (cur or {}).get("spec", {}).get("version", 0) + 1 if isinstance(cur, dict) else 1
    kv.set("jobresource", json.dumps(jr.to_dict()))
    print(json.dumps({"applied_version": jr.version}))


def cmd_scale(a):
    from easydl_amd.api.spec import JobResource
    kv = _kv(a)
    cur = kv.get("jobresource")
    if not cur:
        raise SystemExit("job has no JobResource yet")
    jr = JobResource.from_dict(cur)
    jr.roles["worker"].replicas = a.workers
    jr.version += 1
    jr.resource_updation = []
    kv.set("jobresource", json.dumps(jr.to_dict()))
    print(json.dumps({"workers": a.workers, "version": jr.version}))


def cmd_status(a):
    kv = _kv(a)
    e = kv.counter("rdzv/epoch")
    out = {"epoch": e, "assignment": kv.get(f"rdzv/assign/{e}") if e else None,
           "jobresource": kv.get("jobresource"), "joined": (kv.get_str("rdzv/joined") or "").strip(",").split(",")}
    print(json.dumps(out, indent=1))


def cmd_kill(a):
    kv = _kv(a)
    info = kv.get(f"rdzv/info/{a.node}")
    if not info:
        raise SystemExit(f"unknown node {a.node}")
    import signal
    os.kill(int(info["pid"]), signal.SIGKILL)
    print(json.dumps({"killed": a.node, "pid": info["pid"]}))


def cmd_brain(a):
    from easydl_amd.brain.service import main as bmain
    bmain(["--port", str(a.port)])


def cmd_logs(a):
    """Tail the logs of a job's processes (``<run_dir>/logs/<job>-<role>-<i>.log``) and,
    with --events, its merged event timeline."""
    import glob
    logs = sorted(glob.glob(os.path.join(a.run_dir, "logs", "*.log")))
    if a.name:
        logs = [p for p in logs if os.path.basename(p).startswith(a.name)]
    for p in logs:
        with open(p, errors="replace") as f:
            lines = f.readlines()[-a.tail:]
        print(f"==> {os.path.basename(p)} <==")
        print("".join(lines), end="" if lines and lines[-1].endswith("\n") else "\n")
    if a.events:
        from easydl_amd.utils.events import read_events
        for e in read_events(a.run_dir)[-a.tail:]:
            print(json.dumps(e))
    return 0 if logs or a.events else 1


def cmd_schema(a):
    from easydl_amd.api.schema import SCHEMAS, document
    kinds = [a.kind] if a.kind else sorted(SCHEMAS)
    print(json.dumps({k: document(k) for k in kinds} if len(kinds) > 1 else document(kinds[0]), indent=1))


def cmd_validate(a):
    """Schema-check every document of a spec file (exit 1 on any violation)."""
    from easydl_amd.api.schema import validate
    from easydl_amd.api.spec import load_yaml_docs
    bad = 0
    for i, d in enumerate(load_yaml_docs(a.spec)):
        errs = validate(d)
        print(json.dumps({"doc": i, "kind": d.get("kind"), "ok": not errs, "errors": errs}))
        bad += bool(errs)
    return 1 if bad else 0


def main(argv=None):
    logging.basicConfig(level=logging.INFO, format="%(asctime)s %(name)s %(message)s")
    ap = argparse.ArgumentParser(prog="edl")
    sub = ap.add_subparsers(dest="cmd", required=True)
    s = sub.add_parser("submit")
    s.add_argument("spec")
    s.add_argument("--gpus", default=None)
    s.add_argument("--run-dir", default=None)
    s.add_argument("--master-port", type=int, default=None)
    s.add_argument("--timeout", type=float, default=None)
    s.add_argument("--standby", type=int, default=0, help="warm spare worker processes (hot standby)")
    s.set_defaults(fn=cmd_submit)
    for name, fn in (("apply", cmd_apply), ("status", cmd_status), ("scale", cmd_scale), ("kill", cmd_kill)):
        p = sub.add_parser(name)
        p.add_argument("--job", required=True)
        p.add_argument("--host", default="127.0.0.1")
        p.add_argument("--port", type=int, required=True)
        if name == "apply":
            p.add_argument("spec")
        if name == "scale":
            p.add_argument("--workers", type=int, required=True)
        if name == "kill":
            p.add_argument("--node", required=True)
        p.set_defaults(fn=fn)
    lg = sub.add_parser("logs", help="tail process logs (and events) of a job's run directory")
    lg.add_argument("--run-dir", required=True)
    lg.add_argument("--name", default=None, help="process name prefix, e.g. myjob-worker-1")
    lg.add_argument("--tail", type=int, default=50)
    lg.add_argument("--events", action="store_true")
    lg.set_defaults(fn=cmd_logs)
    sc = sub.add_parser("schema", help="print the JSON Schema of control-plane messages")
    sc.add_argument("kind", nargs="?", default=None)
    sc.set_defaults(fn=cmd_schema)
    v = sub.add_parser("validate", help="schema-check an ElasticJob / JobResource spec file")
    v.add_argument("spec")
    v.set_defaults(fn=cmd_validate)
    b = sub.add_parser("brain")
    b.add_argument("--port", type=int, default=8808)
    b.set_defaults(fn=cmd_brain)
    a = ap.parse_args(argv)
    rc = a.fn(a)
    return rc or 0


if __name__ == "__main__":
    sys.exit(main())
