#!/bin/bash
# Iteration check: GPU parity tests, a short bench (no CPU baseline), stamps. Stops at the first failure.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out
step() {
  local name=$1 to=$2; shift 2
  echo "=== $name"; date
  timeout -k 10 "$to" "$@" > "$R/gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "rc=$rc"; grep -v amdgpu.ids "$R/gpurun_out/$name.log" | tail -${TAILN:-6}
  if [ $rc -ne 0 ]; then echo "STOP after $name (rc=$rc)"; exit $rc; fi
}
TAILN=4 step pytest_gpu 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread
TAILN=1 step bench 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-e2e
if [ -z "$NO_STAMPS" ]; then TAILN=11 step stamps 300 env CASK_LIB_PATH=cask_amd/build/stamps/libcask_scan.so python tools/stamps.py --files 8; fi
