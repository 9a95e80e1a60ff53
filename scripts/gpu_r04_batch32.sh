#!/bin/bash
# round 4, batch 32: 4-rank kill -> shrink -> rejoin with snapshots, after leaving the segment change to the next
# snapshot when one is in flight at the world change; checkpoint GPU tests
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out/ttr_r04_rejoin4c
timeout -k 10 300 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_ckpt_gpu.py \
    > gpurun_out/r04_b32_tests.log 2>&1
EDL_TTR_KEEP=1 EDL_TTR_DIR=gpurun_out/ttr_r04_rejoin4c timeout -k 10 300 python -u bench.py --fault-inject \
    --share-gpu --gpus 4 --layers 4 --seq 4096 --mbs 1 --accum 1 --warmup 3 --steps 10 --ckpt-interval 2 \
    --standby 1 > gpurun_out/r04_b32_rejoin4.log 2>&1
