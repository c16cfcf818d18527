#!/bin/bash
# GPU parity suite, then configs[2] at several values of one tuning knob (KNOB, default CASK_BIG_REC;
# values in VALS, "default" = unset), then a quick headline bench.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out
KNOB=${KNOB:-CASK_BIG_REC}
[ -z "$NOTESTS" ] && { bash tools/gpu_tests.sh || exit $?; }
for b in ${VALS:-default 1024 2048 4096 16384}; do
  if [ "$b" = default ]; then unset $KNOB; else export $KNOB=$b; fi
  timeout -k 10 200 python -u tools/bench_configs.py cfg3 --out gpurun_out/cfg3_b$b.json > gpurun_out/cfg3_b$b.log 2>&1 || { tail -20 gpurun_out/cfg3_b$b.log; exit 1; }
  python -c "
import json;d=json.load(open('gpurun_out/cfg3_b$b.json'));d=d[0] if isinstance(d,list) else d;print('$KNOB=$b',round(d['gibps'],1),d['breakdown_ms'],d['counters'])"
done
unset $KNOB
timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-e2e > gpurun_out/bench_q.log 2>&1
rc=$?; echo "bench rc=$rc"; python -c "
import json;d=json.loads(open('gpurun_out/bench_q.log').read().strip().splitlines()[-1]);print('value',d['value'],'kernel_ms',d['roofline']['kernel_ms_avg'],'frac',d['roofline']['frac'],d['pipeline_breakdown_ms'])"
exit $rc
