#!/bin/bash
# round 4, batch 35: VRAM hand-over / warm-up GPU tests after restoring TunableOp state in the warm-up tests
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_vram_handoff.py \
    tests/test_xgmi_gpu.py -m gpu > gpurun_out/r04_b35_tests.log 2>&1
