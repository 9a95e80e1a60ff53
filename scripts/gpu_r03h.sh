#!/bin/bash
# Round 3: IPC lifetime test (a peer's mapping stays readable after the exporter exits).
set -euo pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread \
  tests/test_xgmi_gpu.py -k "outlives" > gpurun_out/r03h_lifetime.log 2>&1
tail -3 gpurun_out/r03h_lifetime.log
