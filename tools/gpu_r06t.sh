#!/bin/bash
# round 6: the chase's slot rows stored nontemporal (CASK_CHASE_NT=1, build/var_nt) against the
# product: step times (rows checked by tools/ab.py), then one WRITE_SIZE pass each
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out
export TMPDIR=/tmp
V=cask_amd/build/var_nt/libcask_scan.so
timeout -k 10 600 python -u tools/ab.py --rounds 3 --steps 10 --zipf-gib 32 prod=product nt=$V 2>&1 | grep -v amdgpu.ids | tee gpurun_out/r06t_ab.log
rc=${PIPESTATUS[0]}; [ $rc -ne 0 ] && exit $rc
for x in prod:product nt:$V; do
  n=${x%%:*}; l=${x#*:}
  timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE -d "$R/gpurun_out/r06t_w_$n" -o w --output-format csv -- python3 tools/ab.py --child $l --steps 3 --zipf-gib 32 > gpurun_out/r06t_w_$n.log 2>&1
  rc=$?; echo "pmc $n rc=$rc"; [ $rc -ne 0 ] && { tail -5 gpurun_out/r06t_w_$n.log; exit $rc; }
done
exit 0
