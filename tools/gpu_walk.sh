#!/bin/bash
# Walk-mode bring-up: the scan parity tests in both modes, then configs[2] (auto = walk) measured.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest ${TESTS:-tests/test_scan_gpu.py} -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider \
  > gpurun_out/pytest_walk.log 2>&1
rc=$?; tail -5 gpurun_out/pytest_walk.log; echo "pytest rc=$rc"
[ $rc -ne 0 ] && grep -B5 -A40 "FAILED\|Error" gpurun_out/pytest_walk.log | head -150 && exit $rc
timeout -k 10 400 python -u tools/bench_configs.py cfg3 --out gpurun_out/walk_cfg2.json > gpurun_out/walk_cfg2.log 2>&1
rc=$?; tail -c 2500 gpurun_out/walk_cfg2.log; echo "cfg2 rc=$rc"; exit $rc
