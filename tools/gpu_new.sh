#!/bin/bash
# The tests added this round, one pytest process, then the 2-rank bench rehearsal.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_shard_gpu.py tests/test_configs_gpu.py -x -v --timeout 120 --timeout-method thread -p no:cacheprovider \
  > gpurun_out/new.log 2>&1 || { tail -60 gpurun_out/new.log; exit 1; }
grep -E "PASSED|FAILED|passed|failed" gpurun_out/new.log | tail -12
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 \
  bench.py --gpus 2 --steps 3 --warmup 1 --dist-backend gloo --same-device --no-cpu-baseline > gpurun_out/bench_n2.log 2>&1
rc=$?; grep '^{' gpurun_out/bench_n2.log | cut -c1-400; grep -o '"keydir[^,]*,' gpurun_out/bench_n2.log; echo "bench n2 rc=$rc"
