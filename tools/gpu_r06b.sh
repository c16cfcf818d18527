#!/bin/bash
# round 6: walk-mode scan tests on the current build, then an A/B of search variants on configs[2]
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_scan_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r06b_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r06b_tests.log; echo "pytest rc=$rc"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 700 python -u tools/ab.py --rounds ${ROUNDS:-3} --zipf-gib 32 "$@" 2>&1 | grep -v amdgpu.ids | tee gpurun_out/r06b_ab.log
