#!/bin/bash
# Round 3 session 3: unprofiled BERT-large / ResNet-50 throughput + kernel traces of both.
set -u
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
mkdir -p gpurun_out
timeout -k 10 300 python3 benchmarks/train_bench.py --model bert-large --batch 32 --steps 20 --warmup 3 > gpurun_out/bert.log 2>&1 || { tail -20 gpurun_out/bert.log; exit 1; }
grep -h '"metric"' gpurun_out/bert.log
timeout -k 10 300 python3 benchmarks/train_bench.py --model resnet50 --batch 256 --steps 20 --warmup 3 > gpurun_out/resnet.log 2>&1 || { tail -20 gpurun_out/resnet.log; exit 1; }
grep -h '"metric"' gpurun_out/resnet.log
bash scripts/bert_profile.sh && bash scripts/resnet_profile.sh
