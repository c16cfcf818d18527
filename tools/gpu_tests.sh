#!/bin/bash
# GPU parity suite (one pytest process) then a short bench line.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider \
  > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -5 gpurun_out/pytest_gpu.log; echo "pytest rc=$rc"
[ $rc -ne 0 ] && grep -B5 -A40 "FAILED\|Error" gpurun_out/pytest_gpu.log | head -120 && exit $rc
if [ -n "$BENCH" ]; then
  timeout -k 10 400 python -u bench.py $BENCH > gpurun_out/bench.log 2>&1
  rc=$?; tail -3 gpurun_out/bench.log; echo "bench rc=$rc"; exit $rc
fi
