#!/bin/bash
# round 6: engine tests after the merge rework, configs[3] open phases with the merge's own trace,
# and the host merge alone at configs[3]'s block size (52 M records) on the box's threads
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_scan_gpu.py tests/test_shard_gpu.py tests/test_compaction.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r06h_tests.log 2>&1
rc=$?; tail -2 gpurun_out/r06h_tests.log; echo "pytest rc=$rc"; [ $rc -ne 0 ] && { grep -B5 -A40 "FAILED\|Error" gpurun_out/r06h_tests.log | head -100; exit $rc; }
timeout -k 10 300 python -u tools/merge_bench.py 52000000 > gpurun_out/r06h_merge.log 2>&1
rc=$?; cat gpurun_out/r06h_merge.log; echo "merge rc=$rc"; [ $rc -ne 0 ] && exit $rc
CASK_OPEN_TRACE=1 timeout -k 10 500 python -u tools/bench_configs.py openab --files 64 --dir /dev/shm --out gpurun_out/r06h_openab.json > gpurun_out/r06h_openab.log 2>&1
rc=$?; grep -E "^open|device-reduced|keydir merge" gpurun_out/r06h_openab.log; echo "openab rc=$rc"; [ $rc -ne 0 ] && { tail -30 gpurun_out/r06h_openab.log; exit $rc; }
[ -n "$NOBIG" ] && exit 0
timeout -k 10 400 python -u tools/bigkeys_bench.py --gib 8 --out gpurun_out/r06h_bigkeys.json > gpurun_out/r06h_bigkeys.log 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/r06h_bigkeys.log | tail -8; echo "bigkeys rc=$rc"; exit $rc
