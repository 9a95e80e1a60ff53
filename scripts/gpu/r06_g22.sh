set -u -o pipefail
# after the overlap rule: BERT-large default, then the driver's headline command
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python benchmarks/train_bench.py --model bert-large --batch 32 --steps 10 --warmup 3 \
  > gpurun_out/r06_bert_final.json 2> gpurun_out/r06_bert_final.err || exit 1
tail -1 gpurun_out/r06_bert_final.json | cut -c1-200
timeout -k 10 900 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r06_bench_v3.json 2> gpurun_out/r06_bench_v3.err || exit 1
python -c "import json;d=json.loads(open('gpurun_out/r06_bench_v3.json').read().strip().splitlines()[-1]);print(d['value'],d['time_to_recover_s'],d['ttr']['step_s_steady'])"
