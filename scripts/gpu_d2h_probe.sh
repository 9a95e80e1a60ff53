set -u
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
mkdir -p gpurun_out/d2h
timeout -k 10 200 python scripts/d2h_overlap_probe.py side cumask8 cumask16 cumask32 > gpurun_out/d2h/default.log 2>&1; rc=$?; grep env gpurun_out/d2h/default.log; [ $rc -eq 0 ] || exit $rc
HSA_ENABLE_SDMA=1 GPU_FORCE_BLIT_COPY_SIZE=0 timeout -k 10 200 python scripts/d2h_overlap_probe.py side \
  > gpurun_out/d2h/sdma1.log 2>&1; rc=$?; grep env gpurun_out/d2h/sdma1.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv \
  -d gpurun_out/d2h/trace -o p -- python3 scripts/d2h_overlap_probe.py side > gpurun_out/d2h/trace.log 2>&1; rc=$?
grep -c copyBuffer gpurun_out/d2h/trace/p_kernel_trace.csv; wc -l gpurun_out/d2h/trace/p_memory_copy_trace.csv
env | grep -i "^HSA\|^HIP\|^ROC\|^GPU_" > gpurun_out/d2h/env.txt
exit $rc
