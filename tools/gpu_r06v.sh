#!/bin/bash
# round 6, final build: every -m gpu test, smoke(), the default bench line, then the rocprofv3
# kernel trace + PMC traffic passes of the headline (tools/gpu_profile.sh, TAG=r06v)
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread -p no:cacheprovider \
  > gpurun_out/r06v_gpu_suite.log 2>&1 || { grep -E "FAILED|Error|error" gpurun_out/r06v_gpu_suite.log | head -20; tail -40 gpurun_out/r06v_gpu_suite.log; exit 1; }
tail -1 gpurun_out/r06v_gpu_suite.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r06v_smoke.log 2>&1
rc=$?; tail -2 gpurun_out/r06v_smoke.log; [ $rc -ne 0 ] && exit $rc
TAG=r06v bash tools/gpu_profile.sh > gpurun_out/r06v_profile.log 2>&1
rc=$?; grep -E "^===|^rc=|^\{" gpurun_out/r06v_profile.log | cut -c1-300; exit $rc
