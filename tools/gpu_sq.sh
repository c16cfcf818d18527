#!/bin/bash
# SQ counter passes over bench.py for k_scan_chunks: where the waves spend their cycles, VALU and
# LDS utilisation. One rocprofv3 --pmc run per pass (no sys/runtime trace).
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out
export TMPDIR=/tmp
B="bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-e2e"
rm -rf gpurun_out/sq
pass() {
  local tag=$1; shift
  timeout -s KILL 90 rocprofv3 --pmc "$@" -d gpurun_out/sq/$tag -o $tag --output-format csv -- python3 $B > gpurun_out/sq_$tag.log 2>&1 || { echo "pass $tag failed"; tail -5 gpurun_out/sq_$tag.log; exit 1; }
}
pass a GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CU_CYCLES SQ_INSTS_VALU SQ_INST_CYCLES_VALU SQ_INSTS_LDS SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_LDS_UNALIGNED_STALL
pass b GRBM_GUI_ACTIVE SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_INST_CYCLES_VMEM SQ_INSTS_VMEM SQ_ACTIVE_INST_VALU SQ_WAIT_ANY SQ_WAIT_INST_ANY
pass c GRBM_GUI_ACTIVE SQ_WAVES SQ_INSTS_SALU SQ_INSTS_SMEM SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_SALU SQ_LDS_CMD_FIFO_FULL SQ_LDS_DATA_FIFO_FULL SQ_INSTS_BRANCH
python3 tools/sq_summary.py gpurun_out/sq k_scan_chunks
