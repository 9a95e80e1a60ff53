#!/bin/bash
# round 4, batch 26: shared-GPU rejoin slowdown, default path with per-step phases and the aborted engines'
# release times (xgmi_released events)
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out/rejoin_phases
EDL_STEP_PHASES=1 EDL_TTR_KEEP=1 EDL_TTR_DIR=gpurun_out/rejoin_phases timeout -k 10 300 python -u bench.py \
    --fault-inject --share-gpu --gpus 3 --comm auto-gloo --model llama-tiny --seq 2048 --mbs 2 --accum 1 \
    --steps 200 --warmup 2 --fault-step 4 > gpurun_out/r04_b26_phases.log 2>&1
