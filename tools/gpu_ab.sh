#!/bin/bash
# A/B of library builds (NAME=PATH pairs; PATH "product" = cask_amd/libcask_scan.so) on one box.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out
timeout -k 10 900 python -u tools/ab.py --rounds ${ROUNDS:-3} "$@" 2>&1 | grep -v amdgpu.ids
