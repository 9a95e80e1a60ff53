#!/bin/bash
# Round 3: TP tests over the engine (incl. SP with side-stream wgrad), then TP=2 SP A/B
# (2 ranks sharing one GPU, 70B shapes, 2 layers) with the overlap on / off.
set -euo pipefail
mkdir -p gpurun_out/r03k
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread \
  tests/test_xgmi_gpu.py tests/test_tp.py -m gpu -k "tp or llama" > gpurun_out/r03k/tests.log 2>&1
tail -2 gpurun_out/r03k/tests.log
for ov in 1 0; do
  EDL_TP_OVERLAP=$ov timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
    --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --tp 2 --sp --share-gpu --layers 2 \
    --model llama3-70b --seq 4096 --mbs 1 --accum 1 --steps 6 --warmup 2 --comm xgmi-only \
    --out gpurun_out/r03k/tp2_sp_overlap${ov}.json > gpurun_out/r03k/tp2_sp_overlap${ov}.log 2>&1
  python -c "import json;d=json.load(open('gpurun_out/r03k/tp2_sp_overlap${ov}.json'));print('sp overlap=$ov',d['ms_per_step'],d['loss'])"
done
