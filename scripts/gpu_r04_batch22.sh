#!/bin/bash
# round 4, batch 22: Communicator's RCCL data plane on hardware (world 1): collectives + coalesced p2p batch
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -v --timeout 240 --timeout-method thread \
    tests/test_xgmi_gpu.py -k rccl_data_plane > gpurun_out/r04_b22_tests.log 2>&1
