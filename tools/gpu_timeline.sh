#!/bin/bash
# Kernel + memory-copy timeline of a short bench run (no counters): per-kernel stats and the gaps
# between launches, for tools/timeline.py.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${TAG:-tl}
rm -rf gpurun_out/$TAG
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats -d gpurun_out/$TAG -o run --output-format csv -- \
  python3 bench.py --steps ${STEPS:-10} --warmup 2 --no-cpu-baseline --no-e2e > gpurun_out/$TAG.log 2>&1
rc=$?; tail -2 gpurun_out/$TAG.log; echo rc=$rc
find gpurun_out/$TAG -name "*.csv" | head
