#!/bin/bash
# round 4, batch 9: the headline model with snapshots every 2 steps through windows with fault-around prefault;
# then the whole GPU test tier and the smoke test on this round's tree
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
timeout -k 10 400 python -u bench.py --steps 10 --warmup 3 --ckpt-interval 2 > gpurun_out/r04_bench_ckpt_win2.log 2>&1
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
    > gpurun_out/r04_gpu_tier.log 2>&1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r04_smoke.log 2>&1
