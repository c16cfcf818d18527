#!/bin/bash
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out
for G in ${GEOS:-0}; do
  timeout -k 10 300 env CASK_SCAN_GEOMETRY=$G python tools/stamps.py --files 8 > gpurun_out/stamps_g$G.log 2>&1
  rc=$?; echo "geo $G rc=$rc"; grep -v amdgpu.ids gpurun_out/stamps_g$G.log | tail -8
  [ $rc -eq 0 ] || exit $rc
done
