set -u -o pipefail
# kernel statistics of the final tree's headline step (the run that produced profiles/r06_final_kernel_stats.csv
# wrote rocprofv3's default SQLite database; the CSV was exported from its top_kernels view)
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r06_final_prof -o run -- \
  python3 bench.py --steps 3 --warmup 2 --ttr off > gpurun_out/r06_final_prof.json 2> gpurun_out/r06_final_prof.err || exit 1
f=$(find gpurun_out/r06_final_prof -name "*kernel_stats.csv" | head -1); echo "$f"; head -12 "$f" | cut -c1-160
