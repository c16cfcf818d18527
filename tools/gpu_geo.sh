#!/bin/bash
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out
step() {
  local name=$1 to=$2; shift 2
  echo "=== $name"; date
  timeout -k 10 "$to" "$@" > "$R/gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "rc=$rc"; tail -${TAILN:-12} "$R/gpurun_out/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "STOP after $name (rc=$rc)"; exit $rc; fi
  return 0
}
for g in ${GEOS:-0 1 2}; do
  TAILN=3 step dbg_g$g 300 env CASK_SCAN_GEOMETRY=$g python tools/debug_chunks.py 2
done
for g in ${GEOS:-0 1 2}; do
  TAILN=1 step bench_g$g 300 env CASK_SCAN_GEOMETRY=$g python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-e2e
done
step pytest_gpu 900 python -m pytest tests -m gpu -q --maxfail=8 -p no:cacheprovider
