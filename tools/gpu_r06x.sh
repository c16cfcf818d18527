#!/bin/bash
# round 6: the search's backward window (CASK_SW_BACK=2/3: after 2 or 3 forward windows without a
# start, the window before b0 once, its candidates' chains followed from their records' ends)
# against the product; tools/ab.py checks every variant's rows against the generator
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out
timeout -k 10 900 python -u tools/ab.py --rounds 3 --steps 10 --zipf-gib 32 prod=product back2=cask_amd/build/var_back2/libcask_scan.so back3=cask_amd/build/var_back3/libcask_scan.so 2>&1 | grep -v amdgpu.ids | tee gpurun_out/r06x_ab.log
exit ${PIPESTATUS[0]}
