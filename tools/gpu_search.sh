#!/bin/bash
# Run-start search (configs[2]): the search's phase stamps (diagnostic build), the walk-mode tests,
# then configs[2] timings at several run lengths (tools/ab.py, one process per setting).
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out
timeout -k 10 200 python tools/search_stamps.py > gpurun_out/search_stamps.log 2>&1; tail -3 gpurun_out/search_stamps.log
timeout -k 10 400 python -u -m pytest tests/test_scan_gpu.py -k "walk or mixed or zipf or long" -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_chain.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_chain.log; [ $rc -ne 0 ] && { grep -B5 -A30 "FAILED\|Error" gpurun_out/pytest_chain.log | head -80; exit $rc; }
timeout -k 10 900 python -u tools/ab.py --rounds ${ROUNDS:-1} --steps 10 --zipf-gib 32 ${LIBS:-r32=product r16=product@CASK_WALK_RUN=16 r64=product@CASK_WALK_RUN=64} > gpurun_out/ab_search.log 2>&1
rc=$?; cut -c1-330 gpurun_out/ab_search.log; exit $rc
