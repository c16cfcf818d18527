#!/bin/bash
# Bench (no CPU baseline) for each k_scan_chunks geometry in $GEOS, plus a parity test run per geometry.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out
for g in ${GEOS:-0 1}; do
  timeout -k 10 300 env CASK_SCAN_GEOMETRY=$g python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_g$g.log 2>&1
  rc=$?; echo "geo $g pytest rc=$rc"; tail -2 gpurun_out/pytest_g$g.log
  [ $rc -eq 0 ] || exit $rc
  timeout -k 10 300 env CASK_SCAN_GEOMETRY=$g python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-e2e > gpurun_out/bench_g$g.log 2>&1
  rc=$?; echo "geo $g bench rc=$rc"; grep -o '"value": [0-9.]*\|"kernel_ms_avg": [0-9.]*\|"compact_ms": [0-9.]*' gpurun_out/bench_g$g.log | tr '\n' ' '; echo
  [ $rc -eq 0 ] || exit $rc
done
