#!/bin/bash
# Config 4 per GPU: the PS design's cost on ONE GPU at a per-GPU layout --
# 1 parameter server + 1 BERT-large worker sharing GPU 0 (IPC transport, fp32 AdamW on the PS,
# bf16 replica on the worker) -- against the same model's DDP step on that GPU at the same
# per-GPU batch.  BATCHES (default "8 32": config 4's worker batch and the DDP headline batch);
# SNAP = PS updates between in-memory snapshots (20; 0 = none), PIPE = pipelined pushes (1),
# STEPS = worker steps per run (96).
set -uo pipefail
out=gpurun_out/${TAG:-bert_ps_per_gpu}
mkdir -p $out
for B in ${BATCHES:-8 32}; do
  python - $B ${PROF:-0} ${SNAP:-20} ${PIPE:-1} ${STEPS:-96} <<'PY' > $out/job_b$B.yaml
import sys, yaml
from easydl_amd.api.spec import JobResource, Resource, RoleResource, load_specs
job, _ = load_specs("examples/bert_ps.yaml")
b = int(sys.argv[1])
job.env.update({"EDL_BATCH": str(b), "EDL_SAMPLES": str(int(sys.argv[5]) * b + 64), "EDL_SHARD": str(8 * b), "EDL_NUM_PS": "1",
                "EDL_PS_SNAPSHOT_EVERY": sys.argv[3], "EDL_PS_PIPELINE": sys.argv[4]})
if sys.argv[2] == "1":   # PROF=1: kernel stats of both roles (rocprofv3 --kernel-trace --stats)
    job.env["EDL_ROCPROF_ROLES"] = "parameter_server,worker"
jr = JobResource(f"{job.name}-resource", job.name, {
    "parameter_server": RoleResource(1, Resource(gpu=1, cpu=8)),
    "worker": RoleResource(1, Resource(gpu=1, cpu=8))})
print(yaml.safe_dump_all([job.to_dict(), jr.to_dict()]))
PY
  rm -rf $out/run_b$B
  timeout -k 10 400 python -m easydl_amd.cli submit $out/job_b$B.yaml --gpus 0,0 --run-dir $out/run_b$B \
    --timeout 380 > $out/ps_b$B.log 2>&1
  rc=$?; echo "ps batch $B rc=$rc"; [ $rc -eq 0 ] || exit $rc
  [ "${PROF:-0}" = "1" ] && continue
  timeout -k 10 300 python benchmarks/train_bench.py --model bert-large --batch $B --steps 20 --warmup 5 \
    > $out/ddp_b$B.json 2> $out/ddp_b$B.err
  rc=$?; echo "ddp batch $B rc=$rc"; cat $out/ddp_b$B.json; [ $rc -eq 0 ] || exit $rc
done
python - $out <<'PY'
import glob, json, sys
out = sys.argv[1]
rows = []
for run in sorted(glob.glob(f"{out}/run_b*")):
    b = int(run.rsplit("_b", 1)[1])
    ph = []
    for f in glob.glob(f"{run}/events-worker*.jsonl"):
        ph += [json.loads(l) for l in open(f) if '"ps_step_phases"' in l]
    steady = ph[1:] or ph
    step = sum(p["pull_s"] + p["compute_s"] + p["push_s"] for p in steady) / max(1, len(steady))
    try:
        ddp = json.loads([l for l in open(f"{out}/ddp_b{b}.json") if l.startswith("{")][-1])
    except (OSError, IndexError):
        ddp = {}
    rows.append({"batch": b, "ps_samples_per_s": round(b / step, 1) if step else None,
                 "ps_phases": {k: round(sum(p[k] for p in steady) / len(steady), 4) for k in ("pull_s", "compute_s", "push_s")} if steady else None,
                 "ddp_samples_per_s": ddp.get("value"), "windows": len(steady)})
print(json.dumps(rows))
json.dump(rows, open(f"{out}/summary.json", "w"))
PY
