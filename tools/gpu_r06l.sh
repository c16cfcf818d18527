#!/bin/bash
# round 6: rocprofv3 kernel trace of configs[3] opens (the device-reduced keydir's block build)
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out
export TMPDIR=/tmp
CASK_OPEN_TRACE=1 timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/r06l_open" -o kt --output-format csv -- python3 -u tools/open_once.py --files 64 --opens 2 --dir /dev/shm > gpurun_out/r06l_open.log 2>&1
rc=$?; grep -E "^open|device-reduced" gpurun_out/r06l_open.log; echo "rc=$rc"; exit $rc
