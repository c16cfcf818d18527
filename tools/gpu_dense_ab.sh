#!/bin/bash
# GPU parity suite, then the headline loop with each dense-row strategy on one box:
# fused (rows from k_scan_chunks), CASK_DENSE=2 (k_finish launch), CASK_DENSE=0 (repair path + k_compact).
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
  > gpurun_out/pytest_gpu.log 2>&1 || { tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
for k in 1 2; do
for mode in fused 0; do
  if [ $mode = fused ]; then E=""; else E="CASK_DENSE=$mode"; fi
  timeout -k 10 300 env $E python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-e2e --no-segmented > gpurun_out/ab_$mode.log 2>&1 || { tail -5 gpurun_out/ab_$mode.log; exit 1; }
  python -c "
import json;d=json.loads(open('gpurun_out/ab_$mode.log').read().strip().splitlines()[-1])
print('$mode', round(d['value'],1), 'ms/step', round(d['ms_per_step'],4), 'scan', round(d['roofline']['kernel_ms_avg'],4), d['pipeline_breakdown_ms'], d['counters']['dense_path'])"
done
done
