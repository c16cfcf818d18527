#!/bin/bash
# Phase stamps of k_scan_chunks for each library variant in $VARIANTS (cask_amd/build/<v>/).
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out
for V in ${VARIANTS:-stamps}; do
for G in ${GEOS:-0}; do
  timeout -k 10 300 env CASK_LIB_PATH=cask_amd/build/$V/libcask_scan.so CASK_SCAN_GEOMETRY=$G python tools/stamps.py --files 8 > gpurun_out/stamps_${V}_g$G.log 2>&1
  rc=$?; echo "variant $V geo $G rc=$rc"; grep -v amdgpu.ids gpurun_out/stamps_${V}_g$G.log | tail -12
  [ $rc -eq 0 ] || exit $rc
done
done
