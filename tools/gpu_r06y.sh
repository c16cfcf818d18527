#!/bin/bash
# round 6, the final tree: every -m gpu test, smoke(), the default bench line
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread -p no:cacheprovider \
  > gpurun_out/r06y_gpu_suite.log 2>&1 || { grep -E "FAILED|Error|error" gpurun_out/r06y_gpu_suite.log | head -20; tail -40 gpurun_out/r06y_gpu_suite.log; exit 1; }
tail -1 gpurun_out/r06y_gpu_suite.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r06y_smoke.log 2>&1
rc=$?; tail -1 gpurun_out/r06y_smoke.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python bench.py > gpurun_out/r06y_bench.log 2>&1
rc=$?; tail -1 gpurun_out/r06y_bench.log | cut -c1-400; exit $rc
