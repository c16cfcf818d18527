#!/bin/bash
# Walk-mode A/B: the GPU walk-mode tests, then configs[2] under the old grouped path and k_walk_hash
# at each depth (one process per setting, alternating rounds: tools/ab.py).
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out
if [ -z "$NO_TESTS" ]; then
timeout -k 10 ${TTIME:-400} python -u -m pytest ${TESTS:-tests/test_scan_gpu.py} -k "${TK:-walk}" -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
  > gpurun_out/pytest_fused.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_fused.log; echo "pytest rc=$rc"
[ $rc -ne 0 ] && { grep -B5 -A40 "FAILED\|Error" gpurun_out/pytest_fused.log | head -150; exit $rc; }
fi
timeout -k 10 ${ABTIME:-900} python -u tools/ab.py --rounds ${ROUNDS:-2} --steps ${STEPS:-10} --zipf-gib 32 ${LIBS:-old=product@CASK_WALK_FUSED=0 d8=product@CASK_HASH_D=8 d16=product@CASK_HASH_D=16 d32=product@CASK_HASH_D=32} \
  > gpurun_out/ab_fused.log 2>&1
rc=$?; cat gpurun_out/ab_fused.log | cut -c1-400; echo "ab rc=$rc"; exit $rc
