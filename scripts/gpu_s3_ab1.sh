#!/bin/bash
# Session 3 A/B: BERT-large residual-gradient slots (EDL_RESGRAD) and ResNet-50 with MIOpen's
# asm implicit-GEMM NHWC solvers (zero-fill + cast launches around every conv) disabled.
set -u
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
mkdir -p gpurun_out/ab1
timeout -k 10 200 python -u -m pytest tests/test_kernels_gpu.py -k "bert_layer_residual or gelu_mlp" -x -q \
  --timeout 120 --timeout-method thread > gpurun_out/ab1/pytest.log 2>&1 || { tail -30 gpurun_out/ab1/pytest.log; exit 1; }
tail -1 gpurun_out/ab1/pytest.log
for i in 1 2; do
  for rg in 0 1; do
    EDL_RESGRAD=$rg timeout -k 10 200 python3 benchmarks/train_bench.py --model bert-large --batch 32 --steps 20 --warmup 3 > gpurun_out/ab1/bert_rg$rg.log 2>&1 || { tail -20 gpurun_out/ab1/bert_rg$rg.log; exit 1; }
    echo "bert resgrad=$rg $(grep -h '"metric"' gpurun_out/ab1/bert_rg$rg.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
  done
done
timeout -k 10 300 python3 benchmarks/train_bench.py --model resnet50 --batch 256 --steps 20 --warmup 3 > gpurun_out/ab1/rn_default.log 2>&1 || { tail -20 gpurun_out/ab1/rn_default.log; exit 1; }
echo "resnet default $(grep -h '"metric"' gpurun_out/ab1/rn_default.log | cut -c1-120)"
mkdir -p gpurun_out/ab1/miodb_noasm
MIOPEN_USER_DB_PATH=$PWD/gpurun_out/ab1/miodb_noasm MIOPEN_DEBUG_CONV_IMPLICIT_GEMM_ASM_FWD_GTC_XDLOPS_NHWC=0 \
MIOPEN_DEBUG_CONV_IMPLICIT_GEMM_ASM_BWD_GTC_XDLOPS_NHWC=0 MIOPEN_DEBUG_CONV_IMPLICIT_GEMM_ASM_WRW_GTC_XDLOPS_NHWC=0 \
  timeout -k 10 400 python3 benchmarks/train_bench.py --model resnet50 --batch 256 --steps 20 --warmup 3 > gpurun_out/ab1/rn_noasm.log 2>&1 || { tail -20 gpurun_out/ab1/rn_noasm.log; exit 1; }
echo "resnet no-asm-gtc $(grep -h '"metric"' gpurun_out/ab1/rn_noasm.log | cut -c1-160)"
