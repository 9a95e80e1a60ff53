# A/B of the two dK/dV attention kernels (EDL_ATTN_DKDV=32 vs 64) under rocprofv3,
# interleaved twice so clock drift shows.  Also runs the attention numerics tests
# with each variant.  Usage: gpurun -- bash scripts/gpu_attn_ab.sh
set -u
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
mkdir -p gpurun_out/ab
for v in 64 32; do
  EDL_ATTN_DKDV=$v timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread \
    tests/test_attention_gpu.py -m gpu > gpurun_out/ab/test_$v.log 2>&1 || { tail -30 gpurun_out/ab/test_$v.log; exit 1; }
  echo "tests pass with dkdv=$v"
done
for v in 64 32 64 32; do
  export EDL_ATTN_DKDV=$v
  rm -rf gpurun_out/ab/k$v
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/ab/k$v -o a -- python3 scripts/attn_bench.py > gpurun_out/ab/k$v.log 2>&1 || exit $?
  python3 -c "
import csv
for r in csv.DictReader(open('gpurun_out/ab/k$v/a_kernel_stats.csv')):
    if 'attn' in r['Name']: print('dkdv=$v', round(float(r['AverageNs'])/1e3,1), r['Name'][23:70])
"
done
