#!/bin/bash
# round 6: the keydir block build with the rows' fields gathered in sorted order (k_kd_gather):
# shard / engine / collision tests, then the configs[3] open's kernel trace
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest ${TESTS:-tests/test_shard_gpu.py tests/test_scan_gpu.py tests/test_rccl_ranks_gpu.py tests/test_large_configs_gpu.py} -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r06m_tests.log 2>&1
rc=$?; tail -2 gpurun_out/r06m_tests.log; echo "pytest rc=$rc"; [ $rc -ne 0 ] && { grep -B5 -A40 "FAILED\|Error" gpurun_out/r06m_tests.log | head -80; exit $rc; }
CASK_OPEN_TRACE=1 timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/r06m_open" -o kt --output-format csv -- python3 -u tools/open_once.py --files 64 --opens 2 --dir /dev/shm > gpurun_out/r06m_open.log 2>&1
rc=$?; grep -E "^open|device-reduced" gpurun_out/r06m_open.log; echo "rc=$rc"; exit $rc
