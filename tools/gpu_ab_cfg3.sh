#!/bin/bash
# A/B of libraries (NAME=PATH pairs) on one box: headline bench (tools/gpu_ab.sh) then configs[2].
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out
ROUNDS=${ROUNDS:-2} bash tools/gpu_ab.sh "$@" || exit $?
for spec in "$@"; do
  name=${spec%%=*}; lib=${spec#*=}
  CASK_LIB_PATH=$lib timeout -k 10 200 python -u tools/bench_configs.py cfg3 --out gpurun_out/cfg3_$name.json > gpurun_out/cfg3_$name.log 2>&1 || { tail -20 gpurun_out/cfg3_$name.log; exit 1; }
  python -c "
import json;d=json.load(open('gpurun_out/cfg3_$name.json'));d=d[0] if isinstance(d,list) else d;print('cfg3 $name',round(d['gibps'],1),d['breakdown_ms'],d['counters'])"
done
