set -u -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -v --timeout 400 --timeout-method thread -m gpu tests/test_standby_overlap_gpu.py \
  > gpurun_out/r06_g30.log 2>&1
rc=$?; grep -E "passed|failed" gpurun_out/r06_g30.log | tail -2; exit $rc
