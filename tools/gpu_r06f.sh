#!/bin/bash
# round 6: the overlapped walk — walk-mode tests, then A/B against the serial walk on configs[2]
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_scan_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r06f_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r06f_tests.log; echo "pytest rc=$rc"; [ $rc -ne 0 ] && { grep -B5 -A40 "FAILED\|Error" gpurun_out/r06f_tests.log | head -80; exit $rc; }
timeout -k 10 700 python -u tools/ab.py --rounds ${ROUNDS:-2} --zipf-gib 32 overlap=product serial=product@CASK_TEST_HOOKS=1,CASK_WALK_OVERLAP=0 $EXTRA 2>&1 | grep -v amdgpu.ids | tee gpurun_out/r06f_ab.log
