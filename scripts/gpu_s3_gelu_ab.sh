#!/bin/bash
# GELU kernels with a hardware reciprocal in tanh (no IEEE division): numerics,
# then BERT-large A/B against the previous library (abtmp/lib_gelu) and a kernel profile.
set -u
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
mkdir -p gpurun_out/gelu
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/gelu/pytest.log 2>&1 || { tail -30 gpurun_out/gelu/pytest.log; exit 1; }
tail -1 gpurun_out/gelu/pytest.log
BASE=$PWD/abtmp/lib_gelu
for i in 1 2 3; do
  timeout -k 10 200 python3 benchmarks/train_bench.py --model bert-large --batch 32 --steps 20 --warmup 3 \
    > gpurun_out/gelu/new$i.log 2>&1 || { tail gpurun_out/gelu/new$i.log; exit 1; }
  echo "bert new:  $(grep -h '"metric"' gpurun_out/gelu/new$i.log | cut -c45-120)"
  EDL_LIBDIR=$BASE timeout -k 10 200 python3 benchmarks/train_bench.py --model bert-large --batch 32 --steps 20 \
    --warmup 3 > gpurun_out/gelu/base$i.log 2>&1 || { tail gpurun_out/gelu/base$i.log; exit 1; }
  echo "bert base: $(grep -h '"metric"' gpurun_out/gelu/base$i.log | cut -c45-120)"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/gelu/prof -o bert -- \
  python3 benchmarks/train_bench.py --model bert-large --batch 32 --steps 6 --warmup 2 > gpurun_out/gelu/prof.log 2>&1 \
  || { tail gpurun_out/gelu/prof.log; exit 1; }
echo "profile done"
