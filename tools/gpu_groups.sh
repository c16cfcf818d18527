#!/bin/bash
# Walk groups (CASK_WALK_GROUPS) on configs[2]: one process per setting.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out
for g in ${GROUPS_LIST:-1 2 4 8}; do
  CASK_WALK_GROUPS=$g timeout -k 10 300 python -u tools/bench_configs.py cfg3 --steps 3 > gpurun_out/groups_$g.log 2>&1 || exit 1
  echo "groups=$g $(grep -o '"gibps": [0-9.]*\|"ms_per_step": [0-9.]*\|"chunk_scan_ms": [0-9.]*\|"repaired_chunks": [0-9]*' gpurun_out/groups_$g.log | tr '\n' ' ')"
done
