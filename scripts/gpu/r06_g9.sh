set -u -o pipefail
# Same-box A/B of the round-2 tree (8f7fe00, the driver's 23,489 tok/s) against the head, alternating,
# 3 runs each, at the driver's command (N=1, 20 steps after 5 warm-up; the head without its TTR drill).
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
out=gpurun_out/r06_tree_ab.jsonl
: > $out
for i in 1 2 3; do
  (cd abtmp/r02 && timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > ../../gpurun_out/ab_r02_$i.json 2> ../../gpurun_out/ab_r02_$i.err)
  rc=$?; [ $rc -ne 0 ] && { echo "r02 run $i rc=$rc"; exit $rc; }
  python scripts/ab_line.py gpurun_out/ab_r02_$i.json r02-8f7fe00 $i >> $out
  timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --ttr off > gpurun_out/ab_head_$i.json 2> gpurun_out/ab_head_$i.err
  rc=$?; [ $rc -ne 0 ] && { echo "head run $i rc=$rc"; exit $rc; }
  python scripts/ab_line.py gpurun_out/ab_head_$i.json head $i >> $out
  tail -2 $out
done
