#!/bin/bash
# Sharded replay on one GPU: its -m gpu tests, then bench.py's N>1 path rehearsed with 2 ranks on
# cuda:0 (gloo instead of RCCL: one GPU cannot host two RCCL ranks).
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_shard_gpu.py -x -v --timeout 120 --timeout-method thread -p no:cacheprovider \
  > gpurun_out/shard.log 2>&1 || { tail -40 gpurun_out/shard.log; exit 1; }
tail -8 gpurun_out/shard.log
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 \
  bench.py --gpus 2 --steps 3 --warmup 1 --dist-backend gloo --same-device > gpurun_out/bench_n2.log 2>&1
rc=$?; tail -3 gpurun_out/bench_n2.log | cut -c1-3000; echo "bench n2 rc=$rc"
