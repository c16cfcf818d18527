#!/bin/bash
# Time each diagnostic build in $VARIANTS (cask_amd/build/<v>/libcask_scan.so) and the shipped library.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out
timeout -k 10 200 python tools/time_variant.py shipped 2>&1 | grep -v amdgpu.ids || exit 1
for V in $VARIANTS; do
  timeout -k 10 200 env CASK_LIB_PATH=cask_amd/build/$V/libcask_scan.so python tools/time_variant.py $V 2>&1 | grep -v amdgpu.ids || exit 1
done
