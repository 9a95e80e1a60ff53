set -u -o pipefail
# Rehearsal of the driver's N>1 torchrun form on ONE GPU: 2 ranks share GPU 0 (gloo standing in
# for RCCL, which refuses two ranks on one device); llama-tiny, throughput line only
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29531 bench.py --gpus 2 --steps 3 --warmup 1 --model llama-tiny --share-gpu --comm auto-gloo \
  > gpurun_out/r06_torchrun2.json 2> gpurun_out/r06_torchrun2.err
rc=$?; tail -c 700 gpurun_out/r06_torchrun2.json; [ $rc -ne 0 ] && tail -20 gpurun_out/r06_torchrun2.err; exit $rc
