#!/bin/bash
# configs[2] only, libraries (NAME=PATH pairs) alternated ROUNDS times on one box.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out
for k in $(seq 1 ${ROUNDS:-2}); do
for spec in "$@"; do
  name=${spec%%=*}; lib=${spec#*=}
  CASK_LIB_PATH=$lib timeout -k 10 200 python -u tools/bench_configs.py cfg3 --out gpurun_out/cfg3_$name.json > gpurun_out/cfg3_$name.log 2>&1 || { tail -20 gpurun_out/cfg3_$name.log; exit 1; }
  python -c "
import json;d=json.load(open('gpurun_out/cfg3_$name.json'));d=d[0] if isinstance(d,list) else d;b=d['breakdown_ms'];print('cfg3 $name',round(d['gibps'],1),'scan',round(b['chunk_scan_ms'],2),'long',round(b['long_ms'],2),'repair',round(b['repair_ms'],2))"
done
done
