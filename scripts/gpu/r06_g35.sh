set -u -o pipefail
# final-tree headline: the driver's plain N=1 command
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 900 python -u bench.py > gpurun_out/r06_bench_v5.json 2> gpurun_out/r06_bench_v5.err || exit 1
python scripts/ab_line.py gpurun_out/r06_bench_v5.json head-final 1
