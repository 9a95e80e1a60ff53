#!/bin/bash
# Cross-entropy backward from the saved log-sum-exp (EDL_XENT_LSE): numerics, Llama-3-8B step A/B.
set -u
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
mkdir -p gpurun_out/xent
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_tp.py -k "cross_entropy or xent" -x -q \
  --timeout 120 --timeout-method thread > gpurun_out/xent/pytest.log 2>&1 || { tail -30 gpurun_out/xent/pytest.log; exit 1; }
tail -1 gpurun_out/xent/pytest.log
for i in 1 2; do
  for x in 0 1; do
    EDL_XENT_LSE=$x timeout -k 10 300 python3 bench.py --steps 6 --warmup 2 > gpurun_out/xent/l$x.log 2>&1 \
      || { tail -20 gpurun_out/xent/l$x.log; exit 1; }
    echo "llama EDL_XENT_LSE=$x $(grep -h '"metric"' gpurun_out/xent/l$x.log | cut -c150-230)"
  done
done
