set -u -o pipefail
# per-process TunableOp output file: its GPU test + the probe, then the headline bench on that tree
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_features.py \
  tests/test_gemm_nt_gpu.py > gpurun_out/r06_g39.log 2>&1
rc=$?; grep -E "passed|failed|FAILED" gpurun_out/r06_g39.log | tail -4; [ $rc -ne 0 ] && exit $rc
timeout -k 10 900 python -u bench.py > gpurun_out/r06_bench_v6.json 2> gpurun_out/r06_bench_v6.err || exit 1
python scripts/ab_line.py gpurun_out/r06_bench_v6.json head-final 2
