#!/bin/bash
# Engine tests (open, compaction, hints, shards) on the GPU box; stops at the first failure.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out
run() {  # run NAME pytest-args...
  local name=$1; shift
  timeout -k 10 ${TT:-400} python -u -m pytest "$@" -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_$name.log 2>&1
  local rc=$?; echo "$name rc=$rc: $(tail -1 gpurun_out/pytest_$name.log)"
  [ $rc -ne 0 ] && { grep -B5 -A30 "FAILED\|Error" gpurun_out/pytest_$name.log | head -60; exit $rc; }
  return 0
}
run open tests/test_scan_gpu.py -k "engine_open or sharded_fold"
run compaction tests/test_compaction.py
run hints tests/test_hints_gpu.py
run shard tests/test_shard_gpu.py
