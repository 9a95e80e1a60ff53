#!/bin/bash
# Round 3: kill -> shrink -> rejoin drill with the gradient groups now small enough to be
# IPC-mapped (in-place engine all-reduce on registered buffers while a peer dies).
set -euo pipefail
mkdir -p gpurun_out/ttr_j
DRILL_BERT=0 EDL_HANG_DUMP_S=45 EDL_TTR_KEEP=1 EDL_TTR_DIR=gpurun_out/ttr_j timeout -k 10 300 python bench.py \
  --fault-inject --share-gpu --gpus 4 --layers 4 --seq 4096 --mbs 1 --accum 1 --warmup 3 --steps 10 \
  --ckpt-interval 2 --standby 1 > gpurun_out/r03j_ttr_rejoin.json 2> gpurun_out/r03j_ttr_rejoin.err
cat gpurun_out/r03j_ttr_rejoin.json | cut -c1-600
