set -u -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -v -s --timeout 240 --timeout-method thread -m gpu tests/test_graphs_gpu.py \
  > gpurun_out/r06_g25.log 2>&1
rc=$?; grep -E "passed|failed|hip-graph|Error|assert" gpurun_out/r06_g25.log | head -20; exit $rc
