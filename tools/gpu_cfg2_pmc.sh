#!/bin/bash
# configs[2] (32 GiB Zipf) occupancy / stall counters per kernel: the counter list of this box, then
# one rocprofv3 --pmc pass per counter group (each within the per-block slot limits of
# MI355X_MICROARCH.md §rocprofv3 PMC slots), then the kernel-trace stats. Outputs in
# gpurun_out/pmc_<TAG>/; tools/pmc_stall_summary.py turns them into profiles/.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-r03a}
O="$R/gpurun_out/pmc_$TAG"
rm -rf "$O"; mkdir -p "$O"
C="${PMC_CMD:-$R/tools/bench_configs.py cfg3 --steps ${STEPS:-2}}"
timeout -s KILL 60 rocprofv3 -L > "$O/counters.txt" 2>&1 || true
have() { grep -q -w "$1" "$O/counters.txt"; }
pass() {  # pass NAME COUNTER...
  local name=$1; shift
  local use=()
  for c in "$@"; do have "$c" && use+=("$c"); done
  [ ${#use[@]} -eq 0 ] && { echo "skip $name"; return 0; }
  echo "=== $name: ${use[*]}"; date
  timeout -s KILL 300 rocprofv3 --pmc "${use[@]}" -d "$O/$name" -o $name --output-format csv -- python3 $C > "$O/$name.log" 2>&1
  local rc=$?
  echo "rc=$rc"; tail -2 "$O/$name.log"
  [ $rc -ne 0 ] && { echo "STOP after $name"; exit $rc; }
  return 0
}
echo "=== kt"; date
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/kt" -o kt --output-format csv -- python3 $C > "$O/kt.log" 2>&1 || { tail -20 "$O/kt.log"; exit 1; }
tail -1 "$O/kt.log"
pass occ SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU GRBM_GUI_ACTIVE
pass mem SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INSTS_VMEM_WR GRBM_COUNT
pass lds SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SMEM SQ_INST_CYCLES_VMEM_RD SQ_WAIT_INST_ANY SQ_INSTS_VALU_MUL_I32 SQ_ACTIVE_INST_MISC GRBM_GUI_ACTIVE
pass ta TA_BUSY_avr TA_TA_BUSY_sum TCP_TCC_READ_REQ_sum TCC_HIT_sum TCC_MISS_sum
pass tlb TCP_UTCL1_REQUEST_sum TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_UTCL1_THRASHING_STALL_sum GRBM_UTCL2_BUSY GRBM_GUI_ACTIVE
pass tlb2 TCP_UTCL1_STALL_UTCL2_REQ_OUT_OF_CREDITS_sum TCP_UTCL1_TRANSLATION_MISS_UNDER_MISS_sum TCP_UTCL1_STALL_INFLIGHT_MAX_sum TCP_CLIENT_UTCL1_INFLIGHT_sum
if [ -z "$NO_FETCH" ]; then pass fetch FETCH_SIZE; pass write WRITE_SIZE; fi
ls "$O"
