#!/bin/bash
# Diagnostics session: phase stamps, rocprofv3 kernel trace of a short bench, gpu tests.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out
step() {
  local name=$1 to=$2; shift 2
  echo "=== $name"; date
  timeout -k 10 "$to" "$@" > "$R/gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "rc=$rc"; tail -12 "$R/gpurun_out/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "STOP after $name (rc=$rc)"; exit $rc; fi
  return 0
}
step stamps 300 env CASK_LIB_PATH=$R/cask_amd/build/stamps/libcask_scan.so python tools/stamps.py --files 2
export TMPDIR=/tmp
step prof 600 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof -o run --output-format csv -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-e2e
step pytest_gpu 900 python -m pytest tests -m gpu -q --maxfail=8 -p no:cacheprovider
