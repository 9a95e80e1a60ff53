#!/bin/bash
# SiLU's sigmoid with a hardware reciprocal (no IEEE division): numerics, Llama-3-8B step A/B
# against the previous library (abtmp/lib_silu), kernel profile of the new one.
set -u
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
mkdir -p gpurun_out/silu
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/silu/pytest.log 2>&1 || { tail -30 gpurun_out/silu/pytest.log; exit 1; }
tail -1 gpurun_out/silu/pytest.log
BASE=$PWD/abtmp/lib_silu
for i in 1 2; do
  EDL_LIBDIR=$BASE timeout -k 10 300 python3 bench.py --steps 6 --warmup 2 > gpurun_out/silu/base$i.log 2>&1 \
    || { tail gpurun_out/silu/base$i.log; exit 1; }
  echo "llama base: $(grep -h '"metric"' gpurun_out/silu/base$i.log | cut -c150-260)"
  timeout -k 10 300 python3 bench.py --steps 6 --warmup 2 > gpurun_out/silu/new$i.log 2>&1 \
    || { tail gpurun_out/silu/new$i.log; exit 1; }
  echo "llama new:  $(grep -h '"metric"' gpurun_out/silu/new$i.log | cut -c150-260)"
done
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/silu/prof -o bench -- \
  python3 bench.py --steps 3 --warmup 1 > gpurun_out/silu/prof.log 2>&1 || { tail gpurun_out/silu/prof.log; exit 1; }
echo "profile done"
