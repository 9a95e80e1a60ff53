#!/bin/bash
# GPU session: smoke, full GPU test tier, rocprofv3 kernel stats of a short bench.
# Every GPU step has its own time limit; the script stops at the first step that
# crashes or times out.
set -u
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
mkdir -p gpurun_out/prof
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
if [ "${PROF:-1}" = "1" ]; then
  ARGS=${PROF_ARGS:-"--steps 3 --warmup 1"}
  timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o bench -- python3 bench.py $ARGS > gpurun_out/prof/run.log 2>&1
  rc=$?; echo "rocprof rc=$rc"; tail -1 gpurun_out/prof/run.log
fi
exit $rc
