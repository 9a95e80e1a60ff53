#!/bin/bash
# BASELINE config 4 plumbing on ONE MI355X: the Brain's 8-GPU plan for BERT-large
# async PS (2 PS with a 64-CU mask + HBM cap, 6 workers) applied as a JobResource,
# every role sharing GPU 0 (--gpus 0,...,0), PS traffic over the IPC transport.
set -u
mkdir -p gpurun_out
OUT=gpurun_out/bert_ps_1gpu
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
exit $rc
