#!/bin/bash
# rocprofv3 kernel trace of the BERT-large DDP training step (1 GPU) + GPU-busy vs wall analysis.
set -u
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
mkdir -p gpurun_out/bertprof
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/bertprof -o bert -- \
  python3 benchmarks/train_bench.py --model bert-large --batch 32 --steps 10 --warmup 3 ${BERT_ARGS:-} > gpurun_out/bertprof/run.log 2>&1
rc=$?; grep -h '"metric"' gpurun_out/bertprof/run.log; exit $rc
