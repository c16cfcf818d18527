#!/bin/bash
# round 6: compaction A/B — live records gathered on the device (product) against copied out of the
# mapped sources on host threads (build/var_hostcopy: the engine before), at key spaces of 20 % and
# 60 % of the records (configs[3] is 20 %)
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out
for live in 0.2 0.6; do
  for v in dev host; do
    L=""; [ $v = host ] && L="--lib cask_amd/build/var_hostcopy/libcask_scan.so"
    o=gpurun_out/r06p_${v}_$live
    CASK_TEST_HOOKS=1 CASK_COMPACT_TRACE=1 timeout -k 10 400 python -u tools/bench_configs.py compact --files 64 --dir /dev/shm --live $live $L --out $o.json > $o.log 2>&1
    rc=$?; echo "== $v live $live rc=$rc"; grep -E "compact batches" $o.log | cut -c1-220
    python3 -c "import json; d=json.load(open('$o.json'))[0]; print({k: round(d[k], 3) for k in ('open_s', 'compact_s', 'reopen_s', 'live_records')}, {k: round(v, 1) for k, v in d['compact_report'].items() if k.endswith('_ms')}, d['compact_report']['bytes_out'])"
    [ $rc -ne 0 ] && exit $rc
  done
done
exit 0
