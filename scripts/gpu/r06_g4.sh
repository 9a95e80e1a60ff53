set -u -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 200 python -u -m pytest -v --timeout 150 --timeout-method thread -m gpu tests/test_kmix.py -s \
  > gpurun_out/r06_g4_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; [ $rc -ge 124 ] && exit $rc
timeout -k 10 900 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r06_bench_b.json 2> gpurun_out/r06_bench_b.err
echo rc=$?
