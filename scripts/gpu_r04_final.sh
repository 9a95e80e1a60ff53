#!/bin/bash
# round 4, final validation on the final tree: the whole GPU test tier, the smoke test, the headline bench, the
# 3-rank kill -> shrink -> rejoin drill (auto plane, hot standby with VRAM hand-over) and the no-survivor drills:
# a kill inside an update (restore from /dev/shm) and a kill between updates (HBM resume)
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out/final_drill gpurun_out/final_ttr
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
    > gpurun_out/r04_final_gpu_tier.log 2>&1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r04_final_smoke.log 2>&1
timeout -k 10 400 python -u bench.py > gpurun_out/r04_final_bench.log 2>&1
EDL_TTR_KEEP=1 EDL_TTR_DIR=gpurun_out/final_drill timeout -k 10 300 python -u bench.py --fault-inject --share-gpu \
    --gpus 3 --comm auto-gloo --model llama-tiny --seq 2048 --mbs 2 --accum 1 --steps 200 --warmup 2 --fault-step 4 \
    > gpurun_out/r04_final_drill.log 2>&1
EDL_TTR_KEEP=1 EDL_TTR_DIR=gpurun_out/final_ttr timeout -k 10 500 python -u bench.py --fault-inject --gpus 1 \
    --mbs 1 --accum 1 --steps 10 --warmup 7 --fault-step 10 > gpurun_out/r04_final_ttr.log 2>&1
EDL_TTR_KEEP=1 EDL_TTR_DIR=gpurun_out/final_ttr timeout -k 10 400 python -u bench.py --fault-inject --gpus 1 \
    --mbs 1 --accum 1 --steps 12 --warmup 3 --fault-step 4 > gpurun_out/r04_final_ttr_hbm.log 2>&1
