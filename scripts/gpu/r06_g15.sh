set -u -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -v -s --timeout 500 --timeout-method thread -m gpu tests/test_standby_overlap_gpu.py > gpurun_out/r06_g15.log 2>&1
rc=$?; grep -E "passed|failed|ratio" gpurun_out/r06_g15.log; exit $rc
