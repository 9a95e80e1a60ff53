#!/bin/bash
# AdamW grid cap (EDL_ADAMW_GRID) with the optimizer update overlapping the next forward: headline
# throughput (bench.py --ttr off) for caps 2048 (default), 512, 256 on one box.
set -uo pipefail
out=gpurun_out/r05_${TAG:-adamw_grid}; mkdir -p $out
for cap in 2048 512 256 2048; do
  EDL_ADAMW_GRID=$cap timeout -k 10 240 python -u bench.py --ttr off --steps ${STEPS:-10} --warmup 3 \
    > $out/grid$cap.json 2> $out/grid$cap.err || exit 1
  python -c "import json; d=json.loads(open('$out/grid$cap.json').read().splitlines()[-1]); print('cap=$cap', d['value'], d['ms_per_step'])"
done
