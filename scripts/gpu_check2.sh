#!/bin/bash
set -u
mkdir -p gpurun_out
timeout -k 10 300 python -c "import __graft_entry__ as g; g.build(); g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -m pytest tests -m gpu -q -x > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 600 python bench.py --steps 10 --warmup 3 --ckpt-interval 2 > gpurun_out/bench_ckpt.log 2>&1
rc=$?; echo "bench ckpt rc=$rc"; tail -1 gpurun_out/bench_ckpt.log
exit $rc
