set -u -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 900 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r06_bench_v2.json 2> gpurun_out/r06_bench_v2.err
rc=$?; echo "bench rc=$rc"; [ $rc -ne 0 ] && exit $rc
python -c "import json;d=json.loads(open('gpurun_out/r06_bench_v2.json').read().strip().splitlines()[-1]);print(d['value'],d['time_to_recover_s'],d['ttr']['step_s_steady'])"
PROF_ARGS="--steps 3 --warmup 2 --ttr off" bash scripts/gpu/profile.sh
