#!/bin/bash
set -u
mkdir -p gpurun_out
timeout -k 10 400 python -m pytest tests/test_resources_gpu.py tests/test_ckpt_gpu.py -x -q -s > gpurun_out/res_test.log 2>&1
rc=$?; echo "gpu tests rc=$rc"; grep -E "cu-mask|passed|failed|Error" gpurun_out/res_test.log | head -5
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
EDL_TTR_DIR=$PWD/gpurun_out EDL_TTR_KEEP=1 timeout -k 10 900 python bench.py --fault-inject --gpus 1 --steps 5 --warmup 2 --mbs 1 --accum 1 > gpurun_out/ttr.log 2>&1
rc=$?; echo "ttr rc=$rc"; tail -1 gpurun_out/ttr.log
