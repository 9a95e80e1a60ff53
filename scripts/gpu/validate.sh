#!/bin/bash
# Round-end validation on one MI355X, as the driver runs it: the GPU test tier, smoke(), the
# headline bench (throughput child + time-to-recover drill child).  Stops at the first failure.
set -uo pipefail
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
out=gpurun_out/${TAG:-validate}
mkdir -p $out
timeout -k 10 ${TIER_S:-1000} python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
  > $out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1
rc=$?; tail -1 $out/smoke.log; [ $rc -eq 0 ] || exit $rc
[ "${BENCH:-1}" = "1" ] || exit 0
timeout -k 10 900 python -u bench.py > $out/bench.json 2> $out/bench.err
rc=$?; echo "bench rc=$rc"; cat $out/bench.json; exit $rc
