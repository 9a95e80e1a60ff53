#!/bin/bash
# rocprofv3 kernel trace of the ResNet-50 DDP training step (1 GPU, batch 256) + GPU-busy vs wall.
set -u
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
mkdir -p gpurun_out/rnprof
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/rnprof -o rn -- \
  python3 benchmarks/train_bench.py --model resnet50 --batch 256 --steps 10 --warmup 3 > gpurun_out/rnprof/run.log 2>&1
rc=$?; grep -h '"metric"' gpurun_out/rnprof/run.log
[ $rc -eq 0 ] && python3 scripts/step_busy.py gpurun_out/rnprof/rn_kernel_trace.csv > gpurun_out/rnprof/busy.txt && cat gpurun_out/rnprof/busy.txt
exit $rc
