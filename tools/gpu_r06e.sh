#!/bin/bash
# round 6: engine tests, configs[3] open phases (device-reduced vs host fold, open_multi), CU-mask costs
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_scan_gpu.py tests/test_shard_gpu.py tests/test_compaction.py tests/test_rccl_ranks_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r06e_tests.log 2>&1
rc=$?; tail -2 gpurun_out/r06e_tests.log; echo "pytest rc=$rc"; [ $rc -ne 0 ] && { grep -B5 -A40 "FAILED\|Error" gpurun_out/r06e_tests.log | head -100; exit $rc; }
CASK_OPEN_TRACE=1 timeout -k 10 500 python -u tools/bench_configs.py openab --files 64 --dir /dev/shm --out gpurun_out/r06e_openab.json > gpurun_out/r06e_openab.log 2>&1
rc=$?; grep -E "^open|device-reduced" gpurun_out/r06e_openab.log; echo "openab rc=$rc"; [ $rc -ne 0 ] && { tail -30 gpurun_out/r06e_openab.log; exit $rc; }
[ -n "$NOCU" ] && exit 0
T=cask_amd/build/var_tun/libcask_scan.so
timeout -k 10 800 python -u tools/ab.py --rounds 1 --steps 10 --zipf-gib 32 all=$T h240=$T@CASK_HASH_CUS=240 h224=$T@CASK_HASH_CUS=224 h192=$T@CASK_HASH_CUS=192 p128=$T@CASK_PRE_CUS=128 p64=$T@CASK_PRE_CUS=64 p32=$T@CASK_PRE_CUS=32 2>&1 | grep -v amdgpu.ids | tee gpurun_out/r06e_cumask.log
