#!/bin/bash
# A chain of GPU steps for one gpurun call: each "NAME|TIMEOUT|COMMAND" argument runs under its own
# time limit with its output in gpurun_out/NAME.log; the chain stops at the first failure.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out
for spec in "$@"; do
  name=${spec%%|*}; rest=${spec#*|}; to=${rest%%|*}; cmd=${rest#*|}
  echo "=== $name ($to s)"; date
  timeout -k 10 "$to" bash -c "$cmd" > "gpurun_out/$name.log" 2>&1
  rc=$?
  echo "rc=$rc"; tail -${TAILN:-4} "gpurun_out/$name.log" | cut -c1-240
  if [ $rc -ne 0 ]; then echo "STOP after $name (rc=$rc)"; exit $rc; fi
done
