#!/bin/bash
# round 4, batch 25: shared-GPU rejoin slowdown (3 ranks on one GPU, SIGKILL at step 4, standby rejoins):
# default vs no early hand-over vs no VRAM hand-over, to separate the candidates of the open issue
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
run() {
    local name=$1; shift
    mkdir -p gpurun_out/rejoin_$name
    env "$@" EDL_TTR_KEEP=1 EDL_TTR_DIR=gpurun_out/rejoin_$name timeout -k 10 300 python -u bench.py \
        --fault-inject --share-gpu --gpus 3 --comm auto-gloo --model llama-tiny --seq 2048 --mbs 2 --accum 1 \
        --steps 200 --warmup 2 --fault-step 4 > gpurun_out/r04_b25_$name.log 2>&1
}
run default EDL_B25=1
run no_early EDL_EARLY_HANDOVER=0
run no_vram EDL_VRAM_HANDOFF=0
