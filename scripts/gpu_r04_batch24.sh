#!/bin/bash
# round 4, batch 24: PS snapshots through an HBM shadow (the next update no longer waits for the host copy):
# PS GPU tests, then config 4 (BERT-large async PS, 2 PS + 6 workers on one GPU) with and without the shadow
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_ps_sparse.py \
    > gpurun_out/r04_b24_tests.log 2>&1
timeout -k 10 560 bash scripts/bert_ps_1gpu.sh > gpurun_out/r04_b24_bert_ps_shadow.log 2>&1
cp -r gpurun_out/bert_ps_1gpu gpurun_out/bert_ps_1gpu_shadow
EDL_PS_SNAPSHOT_SHADOW=0 timeout -k 10 560 bash scripts/bert_ps_1gpu.sh > gpurun_out/r04_b24_bert_ps_noshadow.log 2>&1
