#!/bin/bash
# configs[2] in walk mode over run lengths and grid sizes (tuning knobs), one process each.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out
for cfg in ${CFGS:-32:16 64:16}; do
  set -- ${cfg/:/ }
  CASK_WALK_RUN=$1 CASK_WALK_WAVES=$2 timeout -k 10 300 python -u tools/bench_configs.py cfg3 --steps 3 > gpurun_out/sweep_$1_$2.log 2>&1 || exit 1
  echo "run=$1 waves=$2 $(grep -o '"ms_per_step": [0-9.]*\|"chunk_scan_ms": [0-9.]*\|"long_ms": [0-9.]*\|"repaired_chunks": [0-9]*' gpurun_out/sweep_$1_$2.log | tr '\n' ' ')"
done
