#!/bin/bash
# round-3 GPU batch: conv op tests, ResNet-50 A/B (1x1 GEMM path), conv probe, Llama bench
set -u -o pipefail
timeout -k 10 300 python -u -m pytest tests/test_conv_ops.py tests/test_xgmi_gpu.py -m gpu -x -q --timeout 240 --timeout-method thread -p no:cacheprovider > gpurun_out/r03c_tests.log 2>&1
echo "tests rc=$?"; tail -2 gpurun_out/r03c_tests.log
for v in 0 1; do
  EDL_CONV1X1_GEMM=$v timeout -k 10 300 python benchmarks/train_bench.py --model resnet50 --batch 256 --steps 20 --warmup 5 > gpurun_out/r03_resnet_gemm$v.json 2> gpurun_out/r03_resnet_gemm$v.err
  echo "resnet gemm=$v rc=$?"; grep metric gpurun_out/r03_resnet_gemm$v.json | cut -c1-200
done
timeout -k 10 200 python scripts/conv1x1_probe.py > gpurun_out/r03_conv1x1_probe.txt 2>&1; tail -1 gpurun_out/r03_conv1x1_probe.txt
timeout -k 10 400 python bench.py --steps 10 --warmup 3 > gpurun_out/r03_bench.json 2> gpurun_out/r03_bench.err
echo "bench rc=$?"; cat gpurun_out/r03_bench.json
