set -u -o pipefail
# HIP-level wait for fresh HBM on a side thread after a recovery: three-failure soak, then the headline bench
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=r06_soak3_regrow bash scripts/gpu/soak_3fail.sh > gpurun_out/r06_soak_regrow.txt 2>&1 || exit 1
timeout -k 10 900 python -u bench.py > gpurun_out/r06_bench_v8.json 2> gpurun_out/r06_bench_v8.err || exit 1
python scripts/ab_line.py gpurun_out/r06_bench_v8.json regrow 1
