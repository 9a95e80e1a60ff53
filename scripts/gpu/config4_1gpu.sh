#!/bin/bash
# BASELINE config 4 plumbing on ONE MI355X: the Brain's 8-GPU plan for BERT-large
# async PS (2 PS with a 64-CU mask + HBM cap, 6 workers) applied as a JobResource,
# every role sharing GPU 0 (--gpus 0,...,0), PS traffic over the IPC transport.
set -u
mkdir -p gpurun_out
OUT=gpurun_out/${TAG:-config4_1gpu}
rm -rf $OUT
python - <<'PY' > /tmp/bert_ps_1gpu.yaml
import yaml
from easydl_amd.api.spec import JobResource, load_specs
from easydl_amd.brain.collectors import GpuInfo, NodeInventory
from easydl_amd.brain.planner import JobFeatures, Planner
from easydl_amd.master.features import extract
job, _ = load_specs("examples/bert_ps.yaml")
inv = NodeInventory(gpus=[GpuInfo(i, "gfx950", 256, 288.0) for i in range(8)], cpus=128, host_mem_gb=2048)
plan = Planner().startup_plan(JobFeatures.from_dict(extract(job)), inv)
job.env.update({"EDL_SAMPLES": "3072", "EDL_SHARD": "64", "EDL_ROCPROF_ROLES": "parameter_server"})
jr = JobResource(f"{job.name}-resource", job.name, plan.roles)
print(yaml.safe_dump_all([job.to_dict(), jr.to_dict()]))
PY
timeout -k 10 500 python -m easydl_amd.cli submit /tmp/bert_ps_1gpu.yaml --gpus 0,0,0,0,0,0,0,0 --run-dir $OUT --timeout 450 > $OUT.log 2>&1
rc=$?
grep -h '"worker_done"\|"startup_plan"\|"ps_step_phases"' $OUT/events-*.jsonl | tail -14
python -c "
import json, sys
from easydl_amd.brain.collectors import rocprof_rank_profiles
from easydl_amd.brain.planner import Planner
p = rocprof_rank_profiles('$OUT')
print(json.dumps({k: dict(v, planned_cu=Planner.cu_for_profile(v)) for k, v in p.items()}))
" > $OUT/rocprof_profiles.json
cat $OUT/rocprof_profiles.json
# steady aggregate: per worker, batch / (pull + compute + push) over its ps_step_phases windows
# after the first one, summed over the workers (profiles/r04_bert_ps_flag_wait.md "Method")
python - $OUT <<'PY'
import glob, json, sys
tot, per = 0.0, {}
for f in sorted(glob.glob(f"{sys.argv[1]}/events-worker*.jsonl")):
    ph = [json.loads(l) for l in open(f) if '"ps_step_phases"' in l][1:]
    if ph:
        step = sum(p["pull_s"] + p["compute_s"] + p["push_s"] for p in ph) / len(ph)
        per[f.rsplit("events-", 1)[1][:-6]] = round(8 / step, 1)
        tot += 8 / step
print(json.dumps({"steady_aggregate_samples_per_s": round(tot, 1), "per_worker": per}))
PY
exit $rc
