#!/bin/bash
# round 4, batch 36: which cache keeps GPU memory after a full-width warm-up (default / TunableOp off / W^T off)
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
timeout -k 10 120 python -u scripts/warm_leak_probe.py > gpurun_out/r04_b36_probe.log 2>&1
EDL_GEMM_TUNING=off timeout -k 10 120 python -u scripts/warm_leak_probe.py >> gpurun_out/r04_b36_probe.log 2>&1
EDL_WT_CACHE=0 timeout -k 10 120 python -u scripts/warm_leak_probe.py >> gpurun_out/r04_b36_probe.log 2>&1
