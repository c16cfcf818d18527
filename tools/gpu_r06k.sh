#!/bin/bash
# round 6: configs[3] end to end — 64 x 1 GiB written to /dev/shm, open() (scan, hint files written,
# keydir reduced on the device), compact_files() of every file, re-open from the hint files — with
# the compaction's phase trace; A/B of this round's engine against the one before the keydir-table
# rework (build/var_old: engine.cpp of 335a321), alternated twice
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out
for r in 0 1; do
  for v in new old; do
    L=""; [ $v = old ] && L="--lib cask_amd/build/var_old/libcask_scan.so"
    CASK_TEST_HOOKS=1 CASK_COMPACT_TRACE=1 CASK_OPEN_TRACE=1 timeout -k 10 600 python -u tools/bench_configs.py compact --files 64 --dir /dev/shm $L --out gpurun_out/r06k_${v}_$r.json > gpurun_out/r06k_${v}_$r.log 2>&1
    rc=$?; echo "== $v round $r rc=$rc"; grep -E "compact hint|compact batches|device-reduced" gpurun_out/r06k_${v}_$r.log | cut -c1-200
    python3 -c "import json; d=json.load(open('gpurun_out/r06k_${v}_$r.json'))[0]; print({k: round(d[k], 3) for k in ('open_s', 'compact_s', 'reopen_s')}, {k: round(v, 1) for k, v in d['compact_report'].items() if k.endswith('_ms')})"
    [ $rc -ne 0 ] && exit $rc
  done
done
for r in 0 1; do
  for v in new old; do
    L=""; [ $v = old ] && L="--lib cask_amd/build/var_old/libcask_scan.so"
    timeout -k 10 300 python -u tools/fold_bench.py --files 16 --reps 3 $L > gpurun_out/r06k_fold_${v}_$r.log 2>&1
    rc=$?; echo "== fold $v round $r rc=$rc"; grep -o '"fold_ms": [0-9.]*' gpurun_out/r06k_fold_${v}_$r.log | tr '\n' ' '; echo
    [ $rc -ne 0 ] && exit $rc
  done
done
exit 0
