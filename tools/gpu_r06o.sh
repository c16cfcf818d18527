#!/bin/bash
# round 6: compaction with the live records read, verified and gathered on the device — the
# compaction tests, the full-size configs[3] compaction against the oracle, then configs[3] end to
# end twice with the phase trace
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_compaction.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r06o_tests.log 2>&1
rc=$?; tail -1 gpurun_out/r06o_tests.log; echo "pytest rc=$rc"; [ $rc -ne 0 ] && { grep -B5 -A40 "FAILED\|Error" gpurun_out/r06o_tests.log | head -80; exit $rc; }
timeout -k 10 500 python -u -m pytest tests/test_large_configs_gpu.py -k cfg3 -m gpu -x -q --timeout 450 --timeout-method thread -p no:cacheprovider > gpurun_out/r06o_large.log 2>&1
rc=$?; tail -1 gpurun_out/r06o_large.log; echo "large rc=$rc"; [ $rc -ne 0 ] && { tail -40 gpurun_out/r06o_large.log; exit $rc; }
for r in 0 1; do
  CASK_TEST_HOOKS=1 CASK_COMPACT_TRACE=1 timeout -k 10 400 python -u tools/bench_configs.py compact --files 64 --dir /dev/shm --out gpurun_out/r06o_cmp_$r.json > gpurun_out/r06o_cmp_$r.log 2>&1
  rc=$?; echo "== round $r rc=$rc"; grep -E "compact hint|compact batches" gpurun_out/r06o_cmp_$r.log | cut -c1-200
  python3 -c "import json; d=json.load(open('gpurun_out/r06o_cmp_$r.json'))[0]; print({k: round(d[k], 3) for k in ('open_s', 'compact_s', 'reopen_s')}, {k: round(v, 1) for k, v in d['compact_report'].items() if k.endswith('_ms')})"
  [ $rc -ne 0 ] && exit $rc
done
exit 0
