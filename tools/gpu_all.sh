#!/bin/bash
# Every -m gpu test in one pytest process (the heavy configs tests last), then the 2-rank bench
# rehearsal on one GPU (gloo), then a short headline bench.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider \
  > gpurun_out/pytest_gpu.log 2>&1 || { grep -E "FAILED|Error|error" gpurun_out/pytest_gpu.log | head -20; tail -60 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
grep -E "test_configs|test_shard" gpurun_out/pytest_gpu.log | tail -12
if [ -z "$NO_N2" ]; then
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 \
  bench.py --gpus 2 --steps 3 --warmup 1 --dist-backend gloo --same-device --no-cpu-baseline > gpurun_out/bench_n2.log 2>&1
rc=$?; grep '^{' gpurun_out/bench_n2.log | cut -c1-300; grep -o '"keydir[^,]*,' gpurun_out/bench_n2.log; echo "bench n2 rc=$rc"
fi
timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/bench.log 2>&1
rc=$?; tail -1 gpurun_out/bench.log | cut -c1-400; echo "bench rc=$rc"
