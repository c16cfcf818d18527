#!/bin/bash
# SQ counter passes over the bench (k_scan_chunks dominant): where do wave cycles go?
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out
export TMPDIR=/tmp
B="$R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-e2e"
rm -rf "$R/gpurun_out/sq"
timeout -k 10 300 rocprofv3 -L > gpurun_out/counters_list.txt 2>&1
grep -o "SQ_[A-Z_0-9]*" gpurun_out/counters_list.txt | sort -u > gpurun_out/sq_counters.txt
wc -l gpurun_out/sq_counters.txt
i=0
for set in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_WAVES" \
           "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS SQ_BUSY_CYCLES SQ_INSTS_SMEM" \
           "SQ_INST_CYCLES_VMEM_RD SQ_INST_CYCLES_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_MISC SQ_INSTS_BRANCH SQ_ACTIVE_INST_FLAT"; do
  i=$((i+1))
  ok=""
  for c in $set; do grep -qx "$c" gpurun_out/sq_counters.txt && ok="$ok $c"; done
  echo "pass $i:$ok"
  timeout -k 10 300 rocprofv3 --pmc $ok -d "$R/gpurun_out/sq/p$i" -o p$i --output-format csv -- python3 $B > gpurun_out/sq_p$i.log 2>&1
  rc=$?; echo "rc=$rc"; [ $rc -eq 0 ] || { tail -5 gpurun_out/sq_p$i.log; exit $rc; }
done
