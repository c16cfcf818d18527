#!/bin/bash
# round 6: keydir block tests, the full-size configs, then the configs[3] open's kernel trace
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_shard_gpu.py tests/test_scan_gpu.py tests/test_rccl_ranks_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r06n_tests.log 2>&1
rc=$?; tail -1 gpurun_out/r06n_tests.log; echo "pytest rc=$rc"; [ $rc -ne 0 ] && { grep -B5 -A40 "FAILED\|Error" gpurun_out/r06n_tests.log | head -80; exit $rc; }
timeout -k 10 700 python -u -m pytest tests/test_large_configs_gpu.py -m gpu -x -v --timeout 600 --timeout-method thread -p no:cacheprovider > gpurun_out/r06n_large.log 2>&1
rc=$?; grep -E "PASS|FAIL|passed|failed" gpurun_out/r06n_large.log | tail -12; echo "large rc=$rc"; [ $rc -ne 0 ] && exit $rc
CASK_TEST_HOOKS=1 CASK_OPEN_TRACE=1 timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/r06n_open" -o kt --output-format csv -- python3 -u tools/open_once.py --files 64 --opens 2 --dir /dev/shm > gpurun_out/r06n_open.log 2>&1
rc=$?; grep -E "^open|device-reduced|keydir merge" gpurun_out/r06n_open.log; echo "rc=$rc"; exit $rc
