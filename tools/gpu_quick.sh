#!/bin/bash
# Quick GPU check: chunk-table probe, GPU tests, bench (no CPU baseline), stamps.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out
step() {
  local name=$1 to=$2; shift 2
  echo "=== $name"; date
  timeout -k 10 "$to" "$@" > "$R/gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "rc=$rc"; grep -v amdgpu.ids "$R/gpurun_out/$name.log" | tail -${TAILN:-6}
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "STOP after $name (rc=$rc)"; exit $rc; fi
  return 0
}
TAILN=4 step probe 300 env CASK_LIB_PATH=cask_amd/build/stamps/libcask_scan.so python tools/probe_persist.py 1 2 3 8
TAILN=3 step pytest_gpu 900 python -m pytest tests -m gpu -q -x -p no:cacheprovider
for g in ${GEOS:-0}; do
  TAILN=1 step bench_g$g 300 env CASK_SCAN_GEOMETRY=$g python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-e2e
  TAILN=7 step stamps_g$g 300 env CASK_SCAN_GEOMETRY=$g python tools/stamps.py --files 8
done
