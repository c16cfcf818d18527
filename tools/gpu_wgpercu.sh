#!/bin/bash
# Chunk-scan time and phase stamps at 1, 2 and 4 resident workgroups per CU (CASK_WG_PER_CU).
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
for w in ${WGS:-1 4}; do
  echo "== WG/CU $w"
  CASK_WG_PER_CU=$w timeout -k 10 200 python tools/time_variant.py wg$w 2>&1 | grep -v amdgpu.ids || exit 1
  CASK_WG_PER_CU=$w CASK_LIB_PATH=cask_amd/build/stamps/libcask_scan.so timeout -k 10 200 python tools/stamps.py --files 8 2>&1 | grep -v amdgpu.ids | tail -11 || exit 1
done
