#!/bin/bash
# GPU parity suite, configs[2] measurement, quick headline bench, configs[2] phase stamps.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out
bash tools/gpu_tests.sh || exit $?
timeout -k 10 300 python -u tools/bench_configs.py cfg3 --out gpurun_out/cfg3.json > gpurun_out/cfg3.log 2>&1
rc=$?; echo "cfg3 rc=$rc"; tail -c 900 gpurun_out/cfg3.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-e2e > gpurun_out/bench_q.log 2>&1
rc=$?; echo "bench rc=$rc"; python -c "
import json;d=json.loads(open('gpurun_out/bench_q.log').read().strip().splitlines()[-1]);print('value',d['value'],'kernel_ms',d['roofline']['kernel_ms_avg'],'frac',d['roofline']['frac'],d['pipeline_breakdown_ms'])"
[ $rc -ne 0 ] && exit $rc
if [ -n "$STAMPS" ]; then
  timeout -k 10 200 python -u tools/stamps.py --zipf-gib 4 > gpurun_out/stz_exact.log 2>&1
  rc=$?; echo "stamps rc=$rc"; grep -v amdgpu.ids gpurun_out/stz_exact.log | tail -13
fi
