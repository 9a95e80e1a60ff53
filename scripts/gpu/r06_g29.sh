set -u -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -v --timeout 400 --timeout-method thread -m gpu tests/test_standby_slab.py \
  tests/test_standby_refill_gpu.py tests/test_standby_overlap_gpu.py tests/test_vram_handoff.py \
  tests/test_second_failure_gpu.py > gpurun_out/r06_g29.log 2>&1
rc=$?; grep -E "passed|failed" gpurun_out/r06_g29.log | tail -3; [ $rc -ne 0 ] && exit $rc
timeout -k 10 900 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r06_bench_v4.json 2> gpurun_out/r06_bench_v4.err || exit 1
python scripts/ab_line.py gpurun_out/r06_bench_v4.json head-final 1
