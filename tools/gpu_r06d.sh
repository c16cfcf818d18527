#!/bin/bash
# round 6: engine tests (device-reduced open, open_multi, compaction), then the full-size configs[3] test
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_scan_gpu.py tests/test_shard_gpu.py tests/test_compaction.py tests/test_hints_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r06d_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r06d_tests.log; echo "pytest rc=$rc"; [ $rc -ne 0 ] && { grep -B5 -A40 "FAILED\|Error" gpurun_out/r06d_tests.log | head -100; exit $rc; }
if [ -n "$LARGE" ]; then
  timeout -k 10 900 python -u -m pytest tests/test_large_configs_gpu.py -k cfg3 -m gpu -x -q -s --timeout 900 --timeout-method thread -p no:cacheprovider > gpurun_out/r06d_large.log 2>&1
  rc=$?; tail -30 gpurun_out/r06d_large.log; echo "large rc=$rc"; exit $rc
fi
