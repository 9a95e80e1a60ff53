#!/bin/bash
# Headline bench as the driver runs it (N=1): throughput child + time-to-recover drill child,
# the drill's run dir kept under gpurun_out/ for the profile.  Then the GPU tests the
# round-5 changes touch (VRAM hand-over, vram/HBM resume).
set -uo pipefail
out=gpurun_out/r05_${1:-bench}
mkdir -p $out/ttr
export EDL_TTR_DIR=$out/ttr EDL_TTR_KEEP=1
timeout -k 10 900 python -u bench.py --steps ${STEPS:-20} --warmup ${WARMUP:-5} > $out/bench.json 2> $out/bench.err
rc=$?
echo "bench rc=$rc"; cat $out/bench.json
[ $rc -eq 0 ] || exit $rc
if [ -n "${TESTS:-}" ]; then
  timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread $TESTS > $out/pytest.log 2>&1
  rc=$?; tail -5 $out/pytest.log; exit $rc
fi
