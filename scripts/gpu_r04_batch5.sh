#!/bin/bash
# round 4, batch 5: no-survivor restore TTR with the restore split into phases (find / open / H2D / checksum /
# finish; the shm unmap moved off the recovery path), the auto-plane rejoin drill with per-step phase events
# (EDL_STEP_PHASES=1: why world 3 ran slowly after the first rejoin in batch 4), config 4 re-measured
# (BERT-large async PS, 2 PS + 6 workers on one GPU) and a rocprofv3 kernel summary of the headline bench
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out/ttr_n1_r5 gpurun_out/ttr_phases
EDL_TTR_KEEP=1 EDL_TTR_DIR=gpurun_out/ttr_n1_r5 timeout -k 10 400 python -u bench.py --fault-inject --gpus 1 \
    --mbs 1 --accum 1 --steps 4 --warmup 3 --fault-step 4 > gpurun_out/r04_ttr_n1_phases.log 2>&1
EDL_STEP_PHASES=1 EDL_TTR_KEEP=1 EDL_TTR_DIR=gpurun_out/ttr_phases timeout -k 10 300 python -u bench.py \
    --fault-inject --share-gpu --gpus 3 --comm auto-gloo --model llama-tiny --seq 2048 --mbs 2 --accum 1 \
    --steps 400 --warmup 2 --fault-step 4 > gpurun_out/r04_drill_phases.log 2>&1
timeout -k 10 580 bash scripts/bert_ps_1gpu.sh > gpurun_out/r04_bert_ps.log 2>&1
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/r04_prof -o r04 -- python bench.py --steps 3 --warmup 2 \
    > gpurun_out/r04_prof_bench.log 2>&1
