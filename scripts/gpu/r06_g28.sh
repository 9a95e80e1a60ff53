set -u -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -v -s --timeout 200 --timeout-method thread -m gpu tests/test_standby_slab.py \
  tests/test_standby_refill_gpu.py > gpurun_out/r06_g28.log 2>&1
rc=$?; grep -E "passed|failed|Error" gpurun_out/r06_g28.log | head; exit $rc
