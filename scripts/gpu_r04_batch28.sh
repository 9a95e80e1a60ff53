#!/bin/bash
# round 4, batch 28: shared-GPU layouts get 2 hardware queues per process (operator): the kill -> shrink -> rejoin
# drill on the default path, then the whole GPU tier and the smoke test
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out/rejoin_fixed
EDL_STEP_PHASES=1 EDL_TTR_KEEP=1 EDL_TTR_DIR=gpurun_out/rejoin_fixed timeout -k 10 300 python -u bench.py \
    --fault-inject --share-gpu --gpus 3 --comm auto-gloo --model llama-tiny --seq 2048 --mbs 2 --accum 1 \
    --steps 200 --warmup 2 --fault-step 4 > gpurun_out/r04_b28_drill.log 2>&1
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
    > gpurun_out/r04_b28_gpu_tier.log 2>&1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r04_b28_smoke.log 2>&1
