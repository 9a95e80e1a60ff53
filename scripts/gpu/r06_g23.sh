set -u -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for b in 8 32; do
  timeout -k 10 240 python -u scripts/graph_probe.py --batch $b > gpurun_out/graph_probe_$b.json 2> gpurun_out/graph_probe_$b.err
  rc=$?; cat gpurun_out/graph_probe_$b.json; [ $rc -ne 0 ] && { tail -20 gpurun_out/graph_probe_$b.err; exit $rc; }
done
exit 0
