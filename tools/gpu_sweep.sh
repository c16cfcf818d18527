#!/bin/bash
# Sweep a tuning environment variable over values: bench (dense + segmented) and stamps each.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out
VAR=${VAR:-CASK_RUN_CHUNKS}
TAILN=3 timeout -k 10 300 env CASK_LIB_PATH=cask_amd/build/stamps/libcask_scan.so python tools/probe_persist.py 2 8 > gpurun_out/probe.log 2>&1 || { echo probe rc=$?; tail -5 gpurun_out/probe.log; exit 1; }
tail -2 gpurun_out/probe.log
for v in ${VALS:-1 4 16 64}; do
  timeout -k 10 300 env $VAR=$v CASK_SCAN_GEOMETRY=${GEO:-0} python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-e2e > gpurun_out/sweep_$v.log 2>&1
  rc=$?; [ $rc -eq 0 ] || { echo "bench $v rc=$rc"; tail -5 gpurun_out/sweep_$v.log; exit $rc; }
  python -c "
import json;d=json.loads(open('gpurun_out/sweep_$v.log').read().strip().splitlines()[-1]);print('$VAR=$v', round(d['value']), 'GiB/s scan_ms', round(d['roofline']['kernel_ms_avg'],3), 'compact', round(d['pipeline_breakdown_ms']['compact_ms'],3), 'seg', round(d['segmented_gibps']))"
  if [ -n "$STAMPS" ]; then
    timeout -k 10 300 env $VAR=$v CASK_SCAN_GEOMETRY=${GEO:-0} python tools/stamps.py --files 8 > gpurun_out/sweep_st_$v.log 2>&1 || exit 1
    grep -v amdgpu gpurun_out/sweep_st_$v.log | tail -8
  fi
done
