#!/bin/bash
# round 4, batch 11: final snapshot path (process-wide mapping, pages allocated + mapped in the background,
# early hand-over): checkpoint + hand-over GPU tests, no-survivor TTR killed late, and the headline model with
# snapshots every 2 steps measured after both slots have been written once (warmup 12)
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out/ttr_n1_r11
timeout -k 10 300 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_ckpt_gpu.py \
    tests/test_vram_handoff.py > gpurun_out/r04_b11_ckpt_tests.log 2>&1
EDL_TTR_KEEP=1 EDL_TTR_DIR=gpurun_out/ttr_n1_r11 timeout -k 10 500 python -u bench.py --fault-inject --gpus 1 \
    --mbs 1 --accum 1 --steps 10 --warmup 7 --fault-step 10 > gpurun_out/r04_ttr_n1_final.log 2>&1
timeout -k 10 500 python -u bench.py --steps 10 --warmup 12 --ckpt-interval 2 > gpurun_out/r04_bench_ckpt_final.log 2>&1
# world-1 steps without the per-step host drain (EDL_STEP_SYNC=1 = the old drain), ResNet-50 (35 ms steps) and the
# headline model
timeout -k 10 400 python -u bench.py --model resnet50 --steps 40 --warmup 10 > gpurun_out/r04_resnet_nosync.log 2>&1
EDL_STEP_SYNC=1 timeout -k 10 400 python -u bench.py --model resnet50 --steps 40 --warmup 10 \
    > gpurun_out/r04_resnet_sync.log 2>&1
timeout -k 10 400 python -u bench.py --steps 10 --warmup 3 > gpurun_out/r04_bench_final.log 2>&1
