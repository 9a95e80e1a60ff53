#!/bin/bash
# round 4, batch 4: config 4 (BERT-large async PS) and the reference's example job (DeepFM CTR) on the GPU
# PS data plane, every role on GPU 0; results under gpurun_out/
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
# config 4 re-measured (BERT-large async PS, 2 PS + 6 workers on one GPU, IPC transport, flag-ordered pushes)
timeout -k 10 580 bash scripts/bert_ps_1gpu.sh > gpurun_out/r04_bert_ps.log 2>&1
# the reference's example job on the GPU data plane, every role on GPU 0 (2 PS + 4 workers + evaluator)
timeout -k 10 400 python -m easydl_amd.cli submit examples/deepctr_ps_gpu.yaml --gpus 0,0,0,0,0,0,0 \
    --run-dir gpurun_out/deepctr_gpu --timeout 360 > gpurun_out/r04_deepctr_gpu.log 2>&1
