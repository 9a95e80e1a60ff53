#!/bin/bash
# round 4, batch 29: config 4 (2 PS + 6 workers on one GPU) with the shared-GPU hardware-queue limit (default now),
# then with HIP's default of 4 queues per process
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 560 bash scripts/bert_ps_1gpu.sh > gpurun_out/r04_b29_bert_ps_hwq2.log 2>&1
rm -rf gpurun_out/bert_ps_1gpu_hwq2 && cp -r gpurun_out/bert_ps_1gpu gpurun_out/bert_ps_1gpu_hwq2
EDL_SHARED_GPU_HW_QUEUES=4 timeout -k 10 560 bash scripts/bert_ps_1gpu.sh > gpurun_out/r04_b29_bert_ps_hwq4.log 2>&1
