#!/bin/bash
# A/B of the headline bench: libraries given as NAME=PATH pairs, alternated ROUNDS times on one box.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out
for k in $(seq 1 ${ROUNDS:-3}); do
  for spec in "$@"; do
    name=${spec%%=*}; lib=${spec#*=}
    CASK_LIB_PATH=$lib timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-e2e --no-segmented \
      > gpurun_out/ab_$name.log 2>&1 || { echo "$name failed"; tail -5 gpurun_out/ab_$name.log; exit 1; }
    python -c "
import json;d=json.loads(open('gpurun_out/ab_$name.log').read().strip().splitlines()[-1])
print('$name', round(d['value'],1), 'kernel_ms', round(d['roofline']['kernel_ms_avg'],4), 'frac', round(d['roofline']['frac'],4), 'pipe', round(d['roofline']['pipeline_ms_avg'],4))"
  done
done
