set -u -o pipefail
# headline command with the HBM gradient shadow forced on (mid-step resume at 2 x 4 micro-batches)
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
EDL_GRAD_SHADOW=force timeout -k 10 900 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r06_bench_shadow.json 2> gpurun_out/r06_bench_shadow.err
rc=$?; echo "bench rc=$rc"; [ $rc -ne 0 ] && { tail -20 gpurun_out/r06_bench_shadow.err; exit $rc; }
python - <<'PY'
import json
d = json.loads(open("gpurun_out/r06_bench_shadow.json").read().strip().splitlines()[-1])
t = d["ttr"]
print(d["value"], d["time_to_recover_s"], t.get("step_s_steady"), t.get("grad_shadow"), t.get("resumed_mid_step"))
fs = t.get("first_step") or {}
print({k: fs.get(k) for k in ("s", "memory_plan", "memory_replans", "pieces")})
PY
