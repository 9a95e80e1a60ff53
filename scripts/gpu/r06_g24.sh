set -u -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -v -s --timeout 300 --timeout-method thread -m gpu tests/test_opt_overlap_gpu.py \
  tests/test_resources_gpu.py > gpurun_out/r06_g24.log 2>&1
rc=$?; grep -E "passed|failed|cu-plan" gpurun_out/r06_g24.log; exit $rc
