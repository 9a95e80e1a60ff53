#!/bin/bash
# GPU tier on one MI355X box: pytest -m gpu, then __graft_entry__.smoke().
# Usage (from the repo root, via gpurun): bash scripts/gpu_tier.sh <tag>
set -eu -o pipefail
tag=${1:-run}
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread -p no:cacheprovider \
  > gpurun_out/${tag}_pytest_gpu.log 2>&1
tail -3 gpurun_out/${tag}_pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${tag}_smoke.log 2>&1
tail -2 gpurun_out/${tag}_smoke.log
