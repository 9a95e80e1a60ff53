set -u -o pipefail
# Bisect the BERT-large regression over round-6 commits: one box, two passes (forward, reverse order)
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
out=gpurun_out/r06_bert_bisect.jsonl
: > $out
run() {
  local t=$1 d=$2 i=$3
  (cd $d && timeout -k 10 300 python benchmarks/train_bench.py --model bert-large --batch 32 --steps 10 --warmup 3 \
    > $GRAFT_REPO_ROOT/gpurun_out/bb_$t.json 2> $GRAFT_REPO_ROOT/gpurun_out/bb_$t.err) || return 1
  python scripts/ab_line.py gpurun_out/bb_$t.json $t $i >> $out
  tail -1 $out
}
trees="r05:abtmp/r05 43f7cd8:abtmp/c_43f7cd8 be02f06:abtmp/c_be02f06 ebf3155:abtmp/c_ebf3155 06b8232:abtmp/c_06b8232 251fc4e:abtmp/c_251fc4e head:."
for p in 1 2; do
  list=$trees
  [ $p -eq 2 ] && list=$(echo $trees | tr ' ' '\n' | tac | tr '\n' ' ')
  for td in $list; do run ${td%%:*} ${td#*:} $p || exit 1; done
done
