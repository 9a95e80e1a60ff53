#!/bin/bash
# round 4: a fresh process's first Llama-3-8B step, cold vs after a 1-layer warm-up of the same width
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
timeout -k 10 300 python -u scripts/first_step_probe.py cold > gpurun_out/r04_first_step_cold.log 2>&1
timeout -k 10 300 python -u scripts/first_step_probe.py warm > gpurun_out/r04_first_step_warm.log 2>&1
