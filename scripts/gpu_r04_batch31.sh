#!/bin/bash
# round 4, batch 31: batch 30 again after serialising the aborted engine release with the next engine build
# per process): Llama-3-8B arch (4 layers, seq 4096) kill 1 of 4 -> shrink -> rejoin with snapshots, and the
# ResNet-50 scale 1 -> 4 mid-run (config 2), 4 ranks sharing one GPU
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out/ttr_r04_rejoin4b
EDL_TTR_KEEP=1 EDL_TTR_DIR=gpurun_out/ttr_r04_rejoin4b timeout -k 10 300 python -u bench.py --fault-inject \
    --share-gpu --gpus 4 --layers 4 --seq 4096 --mbs 1 --accum 1 --warmup 3 --steps 10 --ckpt-interval 2 \
    --standby 1 > gpurun_out/r04_b31_rejoin4.log 2>&1
timeout -k 10 400 python -u bench.py --scale-up 1:4 --steps 40 --warmup 10 > gpurun_out/r04_b31_scaleup.log 2>&1
