#!/bin/bash
# round 4, batch 17: HBM resume (step marks written by the worker's GPU around every optimizer update; a standby
# that adopted the dead worker's HBM resumes from it when no update was in flight): GPU tests, no-survivor TTR
# killed at step 10 and at step 4; full-width standby warm-up; own marks written only after the post-reap check
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out/ttr_n1_r17
timeout -k 10 300 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_ckpt_gpu.py \
    tests/test_vram_handoff.py > gpurun_out/r04_b17_tests.log 2>&1
EDL_TTR_KEEP=1 EDL_TTR_DIR=gpurun_out/ttr_n1_r17 timeout -k 10 500 python -u bench.py --fault-inject --gpus 1 \
    --mbs 1 --accum 1 --steps 10 --warmup 7 --fault-step 10 > gpurun_out/r04_ttr_n1_hbm_r17_late.log 2>&1
EDL_TTR_KEEP=1 EDL_TTR_DIR=gpurun_out/ttr_n1_r17 timeout -k 10 400 python -u bench.py --fault-inject --gpus 1 \
    --mbs 1 --accum 1 --steps 12 --warmup 3 --fault-step 4 > gpurun_out/r04_ttr_n1_hbm_r17_early.log 2>&1
