set -u -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu tests/test_xgmi_gpu.py \
  > gpurun_out/r06_g32.log 2>&1
rc=$?; grep -E "passed|failed|FAILED" gpurun_out/r06_g32.log | tail -4; [ $rc -ne 0 ] && exit $rc
TAG=r06final_world8b bash scripts/gpu/world8_drill.sh > gpurun_out/r06_world8b.txt 2>&1
rc=$?; python -c "
import json; d=json.loads(open('gpurun_out/r05_r06final_world8b/drill.json').read().strip().splitlines()[-1])
print({k: d.get(k) for k in ('value','worlds_seen','time_to_regain_s','steps_lost')}, [ (f['proc'],f['step'],f['world']) for f in d['final_states']][:9])"
exit $rc
