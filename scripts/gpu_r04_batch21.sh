#!/bin/bash
# round 4, batch 21: where the replacement's first step goes after an HBM resume (EDL_STEP_PHASES=1) and what
# the standby's full-width warm-up did (its log line)
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out/ttr_n1_r21
export EDL_PROFILE_FIRST_STEP=1 EDL_STEP_PHASES=1
EDL_TTR_KEEP=1 EDL_TTR_DIR=gpurun_out/ttr_n1_r21 timeout -k 10 400 python -u bench.py \
    --fault-inject --gpus 1 --mbs 1 --accum 1 --steps 12 --warmup 3 --fault-step 4 \
    > gpurun_out/r04_ttr_n1_hbm_r21_phases.log 2>&1
