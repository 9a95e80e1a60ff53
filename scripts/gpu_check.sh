#!/bin/bash
# One GPU-box session: build, smoke, GPU tests, 1-GPU bench.  Stops at the first
# step that crashes/times out (exit codes other than 0/1 from pytest).
set -u
mkdir -p gpurun_out
BENCH_ARGS=${BENCH_ARGS:-"--steps 10 --warmup 3"}
timeout -k 10 300 python -c "import __graft_entry__ as g; g.build(); g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 600 python bench.py $BENCH_ARGS > gpurun_out/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -2 gpurun_out/bench.log
exit $rc
