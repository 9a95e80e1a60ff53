#!/bin/bash
# round 4, batch 34: per-kernel time of the headline step on the final tree (rocprofv3 kernel trace + stats)
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out/prof_final
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_final -o prof --output-format csv \
    -- python3 bench.py --steps 3 --warmup 2 > gpurun_out/r04_b34_prof.log 2>&1
find gpurun_out/prof_final -name "*kernel_stats.csv" | head -3
