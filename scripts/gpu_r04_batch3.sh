#!/bin/bash
# round 4, batch 3: config-3 no-survivor restore TTR on one MI355X (Llama-3-8B, SIGKILL of the only worker,
# hot standby takes over and restores the newest in-memory snapshot), without and with standby pre-mapping
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out/ttr_n1
timeout -k 10 300 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_ckpt_gpu.py \
    > gpurun_out/r04_ckpt_gpu_test.log 2>&1
EDL_TTR_KEEP=1 EDL_TTR_DIR=gpurun_out/ttr_n1 timeout -k 10 400 python -u bench.py --fault-inject --gpus 1 \
    --mbs 1 --accum 1 --steps 4 --warmup 3 --fault-step 4 > gpurun_out/r04_ttr_n1.log 2>&1
EDL_RESTORE_V1=1 EDL_TTR_KEEP=1 EDL_TTR_DIR=gpurun_out/ttr_n1 timeout -k 10 400 python -u bench.py --fault-inject \
    --gpus 1 --mbs 1 --accum 1 --steps 4 --warmup 3 --fault-step 4 > gpurun_out/r04_ttr_n1_restore_v1.log 2>&1
EDL_STANDBY_PREMAP=1 EDL_TTR_KEEP=1 EDL_TTR_DIR=gpurun_out/ttr_n1 timeout -k 10 400 python -u bench.py --fault-inject \
    --gpus 1 --mbs 1 --accum 1 --steps 4 --warmup 3 --fault-step 4 > gpurun_out/r04_ttr_n1_premap.log 2>&1
