#!/bin/bash
# dK/dV kernel variants (exp under the dP chain; straight-line sub-slices below the diagonal):
# numerics tests, then kernel and whole-step A/B against the previous library (abtmp/lib_base).
set -u
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
mkdir -p gpurun_out/dkdv_ab
timeout -k 10 300 python -u -m pytest tests/test_attention_gpu.py -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/dkdv_ab/pytest.log 2>&1 || { tail -30 gpurun_out/dkdv_ab/pytest.log; exit 1; }
tail -1 gpurun_out/dkdv_ab/pytest.log
BASE=$PWD/abtmp/lib_base
for i in 1 2 3; do
  timeout -k 10 120 python3 scripts/attn_time.py || exit 1
  EDL_LIBDIR=$BASE timeout -k 10 120 python3 scripts/attn_time.py || exit 1
done
for i in 1 2; do
  timeout -k 10 300 python3 bench.py --steps 6 --warmup 2 > gpurun_out/dkdv_ab/new$i.log 2>&1 || { tail gpurun_out/dkdv_ab/new$i.log; exit 1; }
  echo "bench new: $(grep -h '"metric"' gpurun_out/dkdv_ab/new$i.log | cut -c150-260)"
  EDL_LIBDIR=$BASE timeout -k 10 300 python3 bench.py --steps 6 --warmup 2 > gpurun_out/dkdv_ab/base$i.log 2>&1 || exit 1
  echo "bench base: $(grep -h '"metric"' gpurun_out/dkdv_ab/base$i.log | cut -c150-260)"
done
