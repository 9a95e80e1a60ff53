#!/bin/bash
# round-3 GPU batch: xGMI tests (staged pull), kill/shrink/rejoin drill, IPC size threshold
set -u -o pipefail
mkdir -p gpurun_out/ttr
timeout -k 10 400 python -u -m pytest tests/test_xgmi_gpu.py -x -v --timeout 240 --timeout-method thread -p no:cacheprovider > gpurun_out/r03b_xgmi.log 2>&1
echo "xgmi tests rc=$?"; tail -3 gpurun_out/r03b_xgmi.log
DRILL_BERT=0 EDL_HANG_DUMP_S=45 EDL_TTR_KEEP=1 EDL_TTR_DIR=gpurun_out/ttr timeout -k 10 300 python bench.py --fault-inject --share-gpu --gpus 4 \
  --layers 4 --seq 4096 --mbs 1 --accum 1 --warmup 3 --steps 10 --ckpt-interval 2 --standby 1 \
  > gpurun_out/r03_ttr_rejoin.json 2> gpurun_out/r03_ttr_rejoin.err
echo "ttr rc=$?"; cat gpurun_out/r03_ttr_rejoin.json
EDL_XGMI_REGISTER_MAX_MB=100000 PROBE_CASES=2:1536:0,2:2040:0,2:2056:0,2:3000:0 timeout -k 10 420 python scripts/diag/ipc_size_probe.py > gpurun_out/r03_ipc_size_probe2.txt 2>&1
echo "probe rc=$?"; cut -c1-160 gpurun_out/r03_ipc_size_probe2.txt
