#!/bin/bash
# open()/compact_files() phases on a configs[3]-shaped database of FILES data files in /dev/shm,
# under each environment setting in KNOBS (space-separated; commas inside one setting), twice.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out
n=0
for rep in 1 2; do
for k in ${KNOBS:-CASK_OPEN_READERS=16}; do
  n=$((n+1))
  env ${k//,/ } timeout -k 10 400 python -u tools/bench_configs.py compact --files ${FILES:-16} --dir /dev/shm --out gpurun_out/open_$n.json > gpurun_out/open_$n.log 2>&1 || { tail -20 gpurun_out/open_$n.log; exit 1; }
  python -c "
import json;d=json.load(open('gpurun_out/open_$n.json'));d=d[-1] if isinstance(d,list) else d
c=d['compact_report']
print('$k open_s', round(d['open_s'],3), {k: round(v) for k, v in d['open_timings_ms'].items()}, 'compact_s', round(d['compact_s'],3), 'gather', round(c['gather_ms']), 'hints', round(c['hints_ms']), 'write', round(c['write_ms']), 'swap', round(c['swap_ms']))"
done
done
