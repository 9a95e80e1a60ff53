#!/bin/bash
# round 4, batch 8: checkpoint + VRAM hand-over GPU tests; no-survivor TTR with windowed snapshot writes (the dying
# worker holds no page tables of its slots), fallocate population and the VRAM hand-over, killed early (step 4)
# and after four snapshots (step 8); the headline model with snapshots every 2 steps through windows
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out/ttr_n1_r8
timeout -k 10 300 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_ckpt_gpu.py \
    tests/test_vram_handoff.py > gpurun_out/r04_b8_ckpt_tests.log 2>&1
EDL_TTR_KEEP=1 EDL_TTR_DIR=gpurun_out/ttr_n1_r8 timeout -k 10 400 python -u bench.py --fault-inject --gpus 1 \
    --mbs 1 --accum 1 --steps 4 --warmup 3 --fault-step 4 > gpurun_out/r04_ttr_n1_win.log 2>&1
EDL_TTR_KEEP=1 EDL_TTR_DIR=gpurun_out/ttr_n1_r8 timeout -k 10 500 python -u bench.py --fault-inject --gpus 1 \
    --mbs 1 --accum 1 --steps 10 --warmup 7 --fault-step 10 > gpurun_out/r04_ttr_n1_win_late.log 2>&1
timeout -k 10 400 python -u bench.py --steps 10 --warmup 3 --ckpt-interval 2 > gpurun_out/r04_bench_ckpt_win.log 2>&1
