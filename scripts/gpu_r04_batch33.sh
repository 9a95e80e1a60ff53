#!/bin/bash
# round 4, batch 33: ResNet-50 elastic scale-up 1 -> 4 mid-run (config 2), 4 ranks sharing one GPU
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
timeout -k 10 400 python -u bench.py --scale-up 1:4 --share-gpu --steps 30 --warmup 10 \
    > gpurun_out/r04_b33_scaleup.log 2>&1
