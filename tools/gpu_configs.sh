#!/bin/bash
# GPU parity suite, then the configs measurements: configs[2] (device-resident scan) and the
# configs[3]-shaped open + compaction on disk (FILES data files of configs[1] records).
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out
df -h /tmp /dev/shm; free -g | head -2
if [ -z "$NO_TESTS" ]; then
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
  > gpurun_out/pytest_gpu.log 2>&1 || { grep -E "FAILED|Error" gpurun_out/pytest_gpu.log | head; tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
fi
timeout -k 10 900 python -u tools/bench_configs.py ${WHAT:-cfg3 compact} --files ${FILES:-4} ${DIR:+--dir $DIR} --out gpurun_out/configs.json > gpurun_out/configs.log 2>&1
rc=$?; tail -c 3000 gpurun_out/configs.log; echo "configs rc=$rc"
