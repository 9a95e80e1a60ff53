#!/bin/bash
# round 4, batch 7: checkpoint + VRAM hand-over GPU tests; no-survivor TTR with the standby adopting the dead
# worker's state buffers (and without, EDL_VRAM_HANDOFF=0); no-survivor restore TTR on the
# default (pageable, staged) snapshot slots; the headline model with snapshots every 2 steps (population started
# at epoch entry); config 4 (BERT-large async PS, 2 PS + 6 workers on one GPU) with the push message sent after
# the flag stores; the DeepFM example job again
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out/ttr_n1_r7
timeout -k 10 300 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_ckpt_gpu.py \
    tests/test_vram_handoff.py > gpurun_out/r04_b7_ckpt_tests.log 2>&1
EDL_TTR_KEEP=1 EDL_TTR_DIR=gpurun_out/ttr_n1_r7 timeout -k 10 400 python -u bench.py --fault-inject --gpus 1 \
    --mbs 1 --accum 1 --steps 4 --warmup 3 --fault-step 4 > gpurun_out/r04_ttr_n1_vram.log 2>&1
EDL_VRAM_HANDOFF=0 EDL_TTR_KEEP=1 EDL_TTR_DIR=gpurun_out/ttr_n1_r7 timeout -k 10 400 python -u bench.py \
    --fault-inject --gpus 1 --mbs 1 --accum 1 --steps 4 --warmup 3 --fault-step 4 > gpurun_out/r04_ttr_n1_staged.log 2>&1
timeout -k 10 400 python -u bench.py --steps 10 --warmup 3 --ckpt-interval 2 > gpurun_out/r04_bench_ckpt_staged.log 2>&1
timeout -k 10 580 bash scripts/bert_ps_1gpu.sh > gpurun_out/r04_bert_ps2.log 2>&1
timeout -k 10 400 python -m easydl_amd.cli submit examples/deepctr_ps_gpu.yaml --gpus 0,0,0,0,0,0,0 \
    --run-dir gpurun_out/deepctr_gpu2 --timeout 360 > gpurun_out/r04_deepctr_gpu2.log 2>&1
