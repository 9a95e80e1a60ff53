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
job.env.update({"EDL_SAMPLES": "12288", "EDL_SHARD": "64", "EDL_ROCPROF_ROLES": "parameter_server"})
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
# steady aggregate: samples of the 16-step ps_step_phases windows that end while EVERY worker is
# still running (from the latest first-window end to the earliest last-window end), divided by that
# span.  Workers claim shards dynamically, so their step counts differ and a sum of per-worker
# rates would count the tail, when fewer workers share the GPU, as if it were concurrent.
python - $OUT <<'PY'
import glob, json, sys
ends = {}
for f in sorted(glob.glob(f"{sys.argv[1]}/events-worker*.jsonl")):
    ends[f] = [json.loads(l)["ts"] for l in open(f) if '"ps_step_phases"' in l]
ends = {f: v for f, v in ends.items() if v}
t0, t1 = max(min(v) for v in ends.values()), min(max(v) for v in ends.values())
n = sum(16 * 8 for v in ends.values() for t in v if t0 < t <= t1)
print(json.dumps({"steady_aggregate_samples_per_s": round(n / (t1 - t0), 1) if t1 > t0 else None,
                  "window_s": round(t1 - t0, 2), "workers": len(ends)}))
PY
exit $rc
