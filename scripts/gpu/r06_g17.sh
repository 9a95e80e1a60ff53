set -u -o pipefail
# round-6 final tree: the other BASELINE models' throughput, then kernel stats of the headline step
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 400 python -u benchmarks/train_bench.py --model bert-large --batch 32 --steps 10 --warmup 3 \
  > gpurun_out/r06_bert.json 2> gpurun_out/r06_bert.err || { tail -5 gpurun_out/r06_bert.err; exit 1; }
tail -1 gpurun_out/r06_bert.json | cut -c1-400
timeout -k 10 400 python -u benchmarks/train_bench.py --model resnet50 --batch 256 --steps 10 --warmup 3 \
  > gpurun_out/r06_resnet.json 2> gpurun_out/r06_resnet.err || { tail -5 gpurun_out/r06_resnet.err; exit 1; }
tail -1 gpurun_out/r06_resnet.json | cut -c1-400
PROF_ARGS="--steps 3 --warmup 2 --ttr off" bash scripts/gpu/profile.sh
