#!/bin/bash
# round 6: cask_keydir_merge_many in the RCCL folds, open_multi and the Python fold — the shard,
# RCCL (stand-in, 2-4 ranks) and scan tests, the full-size configs, the N=2 rehearsal
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_shard_gpu.py tests/test_rccl_ranks_gpu.py tests/test_scan_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r06z_tests.log 2>&1
rc=$?; tail -1 gpurun_out/r06z_tests.log; echo "pytest rc=$rc"; [ $rc -ne 0 ] && { grep -B5 -A40 "FAILED\|Error" gpurun_out/r06z_tests.log | head -80; exit $rc; }
timeout -k 10 700 python -u -m pytest tests/test_large_configs_gpu.py -m gpu -x -q --timeout 600 --timeout-method thread -p no:cacheprovider > gpurun_out/r06z_large.log 2>&1
rc=$?; tail -1 gpurun_out/r06z_large.log; echo "large rc=$rc"; [ $rc -ne 0 ] && { tail -30 gpurun_out/r06z_large.log; exit $rc; }
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 \
  bench.py --gpus 2 --steps 3 --warmup 1 --dist-backend gloo --same-device --no-cpu-baseline > gpurun_out/r06z_bench_n2.log 2>&1
rc=$?; grep '^{' gpurun_out/r06z_bench_n2.log | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); c=d.get('cfg5_shard', {}); print(d['value'], d.get('keydir_ok'), d.get('keydir_gather_fold_ms'), c.get('keydir_ok'), c.get('exchange_fold_ms'), d.get('cfg5_shard_error'))"; echo "bench n2 rc=$rc"; exit $rc
