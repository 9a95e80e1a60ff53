#!/bin/bash
# round 4, batch 3: config-3 no-survivor restore TTR on one MI355X (Llama-3-8B, SIGKILL of the only worker,
# hot standby takes over and restores the newest in-memory snapshot), without and with standby pre-mapping
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out/ttr_n1
EDL_TTR_KEEP=1 EDL_TTR_DIR=gpurun_out/ttr_n1 timeout -k 10 400 python -u bench.py --fault-inject --gpus 1 \
    --mbs 1 --accum 1 --steps 4 --warmup 3 --fault-step 4 > gpurun_out/r04_ttr_n1.log 2>&1
EDL_STANDBY_PREMAP=1 EDL_TTR_KEEP=1 EDL_TTR_DIR=gpurun_out/ttr_n1 timeout -k 10 400 python -u bench.py --fault-inject \
    --gpus 1 --mbs 1 --accum 1 --steps 4 --warmup 3 --fault-step 4 > gpurun_out/r04_ttr_n1_premap.log 2>&1
# config 4 re-measured (BERT-large async PS, 2 PS + 6 workers on one GPU, IPC transport, flag-ordered pushes)
timeout -k 10 580 bash scripts/bert_ps_1gpu.sh > gpurun_out/r04_bert_ps.log 2>&1
# the reference's example job on the GPU data plane, every role on GPU 0 (2 PS + 4 workers + evaluator)
timeout -k 10 400 python -m easydl_amd.cli submit examples/deepctr_ps_gpu.yaml --gpus 0,0,0,0,0,0,0 \
    --run-dir gpurun_out/deepctr_gpu --timeout 360 > gpurun_out/r04_deepctr_gpu.log 2>&1
