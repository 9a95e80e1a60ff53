set -u -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r06_g3_drill
timeout -k 10 400 python -u -m pytest -v --timeout 250 --timeout-method thread -m gpu \
  tests/test_kmix.py tests/test_brain_measured_gpu.py tests/test_ps_failure_gpu.py -s > gpurun_out/r06_g3_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; [ $rc -ge 124 ] && exit $rc
export EDL_FAULT_STEP_MS=2790 EDL_TTR_KEEP=1 EDL_TTR_DIR=gpurun_out/r06_g3_drill
timeout -k 10 500 python bench.py --fault-inject --gpus 1 --model llama3-8b --seq 8192 --mbs 2 --accum 4 \
  --ckpt-interval 2 --standby 1 --fault-mode midstep --fault-step 4 --steps 0 --warmup 0 \
  > gpurun_out/r06_g3_drill.json 2> gpurun_out/r06_g3_drill.err
echo rc=$?
