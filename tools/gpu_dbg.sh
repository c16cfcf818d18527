#!/bin/bash
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out
timeout -k 10 300 env CASK_SCAN_GEOMETRY=0 python tools/debug_chunks.py 2 > gpurun_out/dbg_g0.log 2>&1; echo rc=$?
tail -25 gpurun_out/dbg_g0.log
timeout -k 10 300 env CASK_SCAN_GEOMETRY=1 python tools/debug_chunks.py 2 > gpurun_out/dbg_g1.log 2>&1; echo rc=$?
tail -25 gpurun_out/dbg_g1.log
