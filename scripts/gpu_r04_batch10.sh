#!/bin/bash
# round 4, batch 10: no-survivor TTR with the early hand-over (replacement as soon as the dead worker's address
# space is gone, restored state re-verified after its reap): process-wide snapshot mapping (default) killed early
# and late, per-piece windows killed late; the headline model with snapshots every 2 steps (default mapping)
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out/ttr_n1_r10
EDL_TTR_KEEP=1 EDL_TTR_DIR=gpurun_out/ttr_n1_r10 timeout -k 10 500 python -u bench.py --fault-inject --gpus 1 \
    --mbs 1 --accum 1 --steps 10 --warmup 7 --fault-step 10 > gpurun_out/r04_ttr_n1_early_late.log 2>&1
EDL_TTR_KEEP=1 EDL_TTR_DIR=gpurun_out/ttr_n1_r10 timeout -k 10 400 python -u bench.py --fault-inject --gpus 1 \
    --mbs 1 --accum 1 --steps 4 --warmup 3 --fault-step 4 > gpurun_out/r04_ttr_n1_early.log 2>&1
EDL_SNAPSHOT_WINDOW=1 EDL_TTR_KEEP=1 EDL_TTR_DIR=gpurun_out/ttr_n1_r10 timeout -k 10 500 python -u bench.py \
    --fault-inject --gpus 1 --mbs 1 --accum 1 --steps 10 --warmup 7 --fault-step 10 \
    > gpurun_out/r04_ttr_n1_early_late_win.log 2>&1
timeout -k 10 400 python -u bench.py --steps 10 --warmup 3 --ckpt-interval 2 > gpurun_out/r04_bench_ckpt_map.log 2>&1
