#!/bin/bash
# Optimizer update overlapping the next forward (EDL_OPT_OVERLAP=1) vs serialized, on the headline
# throughput (bench.py --ttr off), alternating runs on one box.
set -uo pipefail
out=gpurun_out/r05_${TAG:-opt_overlap}; mkdir -p $out
for rep in 1 2; do
  for v in 1 0; do
    EDL_OPT_OVERLAP=$v timeout -k 10 240 python -u bench.py --ttr off --steps ${STEPS:-10} --warmup 3 \
      > $out/ovl${v}_$rep.json 2> $out/ovl${v}_$rep.err || exit 1
    python -c "import json,sys; d=json.loads(open('$out/ovl${v}_$rep.json').read().splitlines()[-1]); print('overlap=$v', d['value'], d['ms_per_step'])"
  done
done
