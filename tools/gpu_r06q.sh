#!/bin/bash
# round 6: every -m gpu test, the 2-rank rehearsal on one GPU (gloo), then the default bench line
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider \
  > gpurun_out/r06q_gpu_suite.log 2>&1 || { grep -E "FAILED|Error|error" gpurun_out/r06q_gpu_suite.log | head -20; tail -40 gpurun_out/r06q_gpu_suite.log; exit 1; }
tail -1 gpurun_out/r06q_gpu_suite.log
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 \
  bench.py --gpus 2 --steps 3 --warmup 1 --dist-backend gloo --same-device --no-cpu-baseline > gpurun_out/r06q_bench_n2.log 2>&1
rc=$?; grep '^{' gpurun_out/r06q_bench_n2.log | cut -c1-300; grep -o '"keydir_ok[^,]*,' gpurun_out/r06q_bench_n2.log; echo "bench n2 rc=$rc"
timeout -k 10 400 python bench.py > gpurun_out/r06q_bench.log 2>&1
rc=$?; tail -1 gpurun_out/r06q_bench.log | cut -c1-600; echo "bench rc=$rc"; exit $rc
