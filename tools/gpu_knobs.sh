#!/bin/bash
# configs[2] under environment settings, one process each: KNOBS="A=1,B=2 A=3" (comma-separated per run).
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out
n=0
for k in ${KNOBS:-CASK_WALK_GROUPS=4}; do
  n=$((n+1))
  env ${k//,/ } timeout -k 10 300 python -u tools/bench_configs.py cfg3 --steps 3 > gpurun_out/knobs_$n.log 2>&1 || exit 1
  echo "$k $(grep -o '"gibps": [0-9.]*\|"ms_per_step": [0-9.]*\|"repaired_chunks": [0-9]*' gpurun_out/knobs_$n.log | tr '\n' ' ')"
done
