#!/bin/bash
# round 6: keydir block scratch aliased + released — shard/scan/rccl tests, the N=2 same-device
# rehearsal (cfg5 secondary included), then the configs[3] open's kernel trace
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_shard_gpu.py tests/test_scan_gpu.py tests/test_rccl_ranks_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r06r_tests.log 2>&1
rc=$?; tail -1 gpurun_out/r06r_tests.log; echo "pytest rc=$rc"; [ $rc -ne 0 ] && { grep -B5 -A40 "FAILED\|Error" gpurun_out/r06r_tests.log | head -80; exit $rc; }
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 \
  bench.py --gpus 2 --steps 3 --warmup 1 --dist-backend gloo --same-device --no-cpu-baseline > gpurun_out/r06r_bench_n2.log 2>&1
rc=$?; grep '^{' gpurun_out/r06r_bench_n2.log | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], {k: d[k] for k in d if k.startswith('keydir') or k.startswith('cfg5')})" | cut -c1-1200; echo "bench n2 rc=$rc"; [ $rc -ne 0 ] && exit $rc
CASK_TEST_HOOKS=1 CASK_OPEN_TRACE=1 timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/r06r_open" -o kt --output-format csv -- python3 -u tools/open_once.py --files 64 --opens 2 --dir /dev/shm > gpurun_out/r06r_open.log 2>&1
rc=$?; grep -E "^open|device-reduced" gpurun_out/r06r_open.log; echo "rc=$rc"; exit $rc
