set -u -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -v -s --timeout 300 --timeout-method thread -m gpu \
  tests/test_brain_measured_gpu.py tests/test_kmix.py tests/test_opt_overlap_gpu.py > gpurun_out/r06_g11_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "passed|failed|\[cu-probe\]|\[brain-measured\] plan" gpurun_out/r06_g11_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 900 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r06_bench_v1.json 2> gpurun_out/r06_bench_v1.err
rc=$?; echo "bench rc=$rc"; tail -c 600 gpurun_out/r06_bench_v1.json; exit $rc
