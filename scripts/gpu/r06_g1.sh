set -u -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -v --timeout 150 --timeout-method thread -m gpu tests/test_opt_overlap_gpu.py tests/test_recompute_gpu.py > gpurun_out/r06_g1_tests.log 2>&1 && \
timeout -k 10 900 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r06_bench_a.json 2> gpurun_out/r06_bench_a.err
echo rc=$?
