#!/bin/bash
# Round 3: xGMI engine tests after the per-instance one-shot switch, and the one-shot /
# in-place / staged crossover at latency-bound sizes (ranks sharing one GPU).
set -euo pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_xgmi_gpu.py \
  > gpurun_out/r03e_xgmi_tests.log 2>&1
timeout -k 10 300 python -u scripts/xgmi_microbench.py --ranks 2 4 --mb 0.25 1 4 16 --iters 50 \
  --out gpurun_out/r03e_oneshot_crossover.jsonl > gpurun_out/r03e_microbench.log 2>&1
tail -3 gpurun_out/r03e_xgmi_tests.log
