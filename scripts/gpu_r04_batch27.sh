#!/bin/bash
# round 4, batch 27: shared-GPU rejoin slowdown, hardware-queue oversubscription test: 2 HW queues per process
# (fewer queues than the scheduler maps at once) and no standby warm-up (one stream fewer in the replacement)
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
run() {
    local name=$1; shift
    mkdir -p gpurun_out/rejoin_$name
    env "$@" EDL_STEP_PHASES=1 EDL_TTR_KEEP=1 EDL_TTR_DIR=gpurun_out/rejoin_$name timeout -k 10 300 python -u \
        bench.py --fault-inject --share-gpu --gpus 3 --comm auto-gloo --model llama-tiny --seq 2048 --mbs 2 \
        --accum 1 --steps 200 --warmup 2 --fault-step 4 > gpurun_out/r04_b27_$name.log 2>&1
}
run hwq2 GPU_MAX_HW_QUEUES=2
run nowarm EDL_STANDBY_WARMUP=0
