set -u -o pipefail
# standby warm-up at the split-piece shape: its GPU test, then the three-failure soak (slab on)
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_vram_handoff.py \
  > gpurun_out/r06_g37.log 2>&1
rc=$?; grep -E "passed|failed|FAILED" gpurun_out/r06_g37.log | tail -4; [ $rc -ne 0 ] && exit $rc
TAG=r06_soak3_piece bash scripts/gpu/soak_3fail.sh > gpurun_out/r06_soak_piece.txt 2>&1
rc=$?; tail -c 300 gpurun_out/r06_soak_piece.txt; exit $rc
