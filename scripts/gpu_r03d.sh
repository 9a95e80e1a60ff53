#!/bin/bash
# Llama-3-8B bench twice on one box (variance) + rocprof kernel stats of a short run
set -u -o pipefail
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
for i in 1 2; do
  timeout -k 10 400 python bench.py --steps 10 --warmup 3 > gpurun_out/r03_bench_$i.json 2> gpurun_out/r03_bench_$i.err
  echo "bench $i rc=$?"; python -c "import json;d=json.load(open('gpurun_out/r03_bench_$i.json'));print(d['value'],d['ms_per_step'])"
done
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r03_prof -o llama -- python3 bench.py --steps 3 --warmup 1 > gpurun_out/r03_prof.log 2>&1
echo "prof rc=$?"; ls gpurun_out/r03_prof | head
