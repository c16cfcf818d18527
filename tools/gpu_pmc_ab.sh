#!/bin/bash
# PMC passes over one configs[2] child of tools/ab.py per library build (NAME=PATH ...): memory-side
# read requests, L2 hits/misses and the wave-cycle split, one rocprofv3 --pmc pass per group.
# Outputs in gpurun_out/pmcab_<TAG>/<NAME>_<pass>/; tools/rdreq_summary.py-style CSVs.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-r04}
O="$R/gpurun_out/pmcab_$TAG"
rm -rf "$O"; mkdir -p "$O"
P=(
  "req TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum"
  "hit TCC_HIT_sum TCC_MISS_sum"
  "occ SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU"
)
for spec in "$@"; do
  name=${spec%%=*}; lib=${spec#*=}
  envs=()
  if [[ "$lib" == *@* ]]; then  # NAME=PATH@VAR=VALUE[,VAR=VALUE]: that build's environment
    IFS=',' read -ra envs <<< "${lib#*@}"; lib=${lib%%@*}
  fi
  for p in "${P[@]}"; do
    set -- $p; pn=$1; shift
    echo "=== $name $pn"; date
    env "${envs[@]}" timeout -s KILL 300 rocprofv3 --pmc "$@" -d "$O/${name}_$pn" -o ${name}_$pn --output-format csv -- \
      python3 tools/ab.py --child "$lib" --steps 3 --zipf-gib 32 > "$O/${name}_$pn.log" 2>&1
    rc=$?
    echo "rc=$rc"; tail -1 "$O/${name}_$pn.log" | cut -c1-160
    [ $rc -ne 0 ] && { echo "STOP"; exit $rc; }
  done
done
exit 0
