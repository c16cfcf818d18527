#!/bin/bash
# k_scan_chunks phase stamps on configs[2]-shaped files, speculative pass only (CASK_NO_REPAIR).
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out
CASK_NO_REPAIR=1 CASK_LIB_PATH=cask_amd/build/stamps/libcask_scan.so timeout -k 10 200 python -u tools/stamps.py --zipf-gib 4 > gpurun_out/stz1.log 2>&1
rc=$?; echo "stamps rc=$rc"; grep -v amdgpu.ids gpurun_out/stz1.log | tail -14; exit $rc
