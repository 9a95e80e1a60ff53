set -u -o pipefail
# allocator pre-growth on a side thread after a recovery: three-failure soak, then the headline bench
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=r06_soak3_pregrow bash scripts/gpu/soak_3fail.sh > gpurun_out/r06_soak_pregrow.txt 2>&1 || exit 1
timeout -k 10 900 python -u bench.py > gpurun_out/r06_bench_v7.json 2> gpurun_out/r06_bench_v7.err || exit 1
python scripts/ab_line.py gpurun_out/r06_bench_v7.json pregrow 1
