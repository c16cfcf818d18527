#!/bin/bash
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out
for rd in 8 16 8 16; do
  CASK_OPEN_READERS=$rd timeout -k 10 400 python -u tools/bench_configs.py compact --files 16 --dir /dev/shm --out gpurun_out/open_$rd.json > gpurun_out/open_$rd.log 2>&1 || { tail -20 gpurun_out/open_$rd.log; exit 1; }
  python -c "
import json;d=json.load(open('gpurun_out/open_$rd.json'));d=d[-1] if isinstance(d,list) else d
print('readers $rd open_s', round(d['open_s'],3), d['open_timings_ms'], 'compact_s', round(d['compact_s'],3))"
done
