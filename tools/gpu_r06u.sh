#!/bin/bash
# round 6: fresh keydir table pages faulted in order before the inserts (product) against faulted by
# the inserts (build/var_nopf): the 52 M-record merge alone, alternated, then the host fold bench
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out
V=cask_amd/build/var_nopf/libcask_scan.so
for r in 0 1; do
  for v in pf nopf; do
    L=""; [ $v = nopf ] && L=$V
    echo "== merge $v round $r"; timeout -k 10 300 python -u tools/merge_bench.py 52000000 $L 2>&1 | grep -E "tables|records:" || exit 1
  done
done
for r in 0 1; do
  for v in pf nopf; do
    L=""; [ $v = nopf ] && L="--lib $V"
    echo "== fold $v round $r"; timeout -k 10 300 python -u tools/fold_bench.py --files 16 --reps 3 $L 2>&1 | grep -o '"fold_ms": [0-9.]*' | tr '\n' ' '; echo
  done
done
exit 0
