#!/bin/bash
# rocprofv3 kernel-trace + stats of a short 1-GPU bench run (no PMC counters here).
set -u
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
mkdir -p gpurun_out/prof
ARGS=${PROF_ARGS:-"--steps 2 --warmup 1"}
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o bench -- python3 bench.py $ARGS > gpurun_out/prof/run.log 2>&1
rc=$?; echo "rocprof rc=$rc"; tail -2 gpurun_out/prof/run.log
find gpurun_out/prof -name "*stats*" | head
exit $rc
