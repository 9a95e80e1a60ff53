#!/bin/bash
# ResNet-50 A/B: MIOpen's asm implicit-GEMM NHWC solvers (a zero-fill launch before every conv,
# plus a cast after the fp32-workspace ones) vs MIOpen with those solvers disabled (fresh find).
set -u
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
mkdir -p gpurun_out/ab1/miodb_noasm
rn() {  # $1 = label
  timeout -k 10 400 python3 benchmarks/train_bench.py --model resnet50 --batch 256 --steps 20 --warmup 3 \
    > gpurun_out/ab1/rn_$1.log 2>&1 || { tail -20 gpurun_out/ab1/rn_$1.log; return 1; }
  echo "resnet $1 $(grep -h '"metric"' gpurun_out/ab1/rn_$1.log | cut -c1-160)"
}
rn default || exit 1
export MIOPEN_USER_DB_PATH=$PWD/gpurun_out/ab1/miodb_noasm
export MIOPEN_DEBUG_CONV_IMPLICIT_GEMM_ASM_FWD_GTC_XDLOPS_NHWC=0
export MIOPEN_DEBUG_CONV_IMPLICIT_GEMM_ASM_BWD_GTC_XDLOPS_NHWC=0
export MIOPEN_DEBUG_CONV_IMPLICIT_GEMM_ASM_WRW_GTC_XDLOPS_NHWC=0
rn noasm || exit 1
rn noasm_again || exit 1
