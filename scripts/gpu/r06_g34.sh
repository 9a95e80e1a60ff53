set -u -o pipefail
# reduced-width standby warm-up: its GPU test, then the three-failure soak (slab on, the default)
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_vram_handoff.py \
  > gpurun_out/r06_g34.log 2>&1
rc=$?; grep -E "passed|failed|FAILED" gpurun_out/r06_g34.log | tail -4; [ $rc -ne 0 ] && exit $rc
TAG=r06_soak3_reduced bash scripts/gpu/soak_3fail.sh > gpurun_out/r06_soak_reduced.txt 2>&1
rc=$?; tail -c 300 gpurun_out/r06_soak_reduced.txt; exit $rc
