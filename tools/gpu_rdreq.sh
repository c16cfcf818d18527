#!/bin/bash
# Round 4: where k_run_hash's counter traffic above the log bytes comes from. One rocprofv3 --pmc pass
# per counter pair (memory-side read requests by size, L2 hits/misses, DRAM-side requests) over
#   * tools/ubench_quads o: the quad access pattern with record bodies at +4 (rounds share a line), at
#     +0 (128-B aligned rounds) and at +64, on a known byte count (the calibration), and
#   * bench.py on configs[2] (the headline's k_run_hash).
# Outputs in gpurun_out/rdreq_<TAG>/; tools/rdreq_summary.py turns them into profiles/.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-r04a}
O="$R/gpurun_out/rdreq_$TAG"
rm -rf "$O"; mkdir -p "$O"
B="$R/bench.py --steps ${PSTEPS:-4} --warmup 1 --no-cpu-baseline --no-e2e --no-cfg1 --no-shard-n1"
run() {  # run NAME TIMEOUT CMD...
  local name=$1 to=$2; shift 2
  echo "=== $name"; date
  timeout -s KILL "$to" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  echo "rc=$rc"; tail -2 "$O/$name.log"
  [ $rc -ne 0 ] && { echo "STOP after $name"; exit $rc; }
  return 0
}
run ubench 120 ./tools/ubench_quads o
P=(
  "req TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum"
  "req2 TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum"
  "hit TCC_HIT_sum TCC_MISS_sum"
  "dram TCC_EA0_RDREQ_DRAM_sum TCC_READ_sum"
)
for p in "${P[@]}"; do
  set -- $p; name=$1; shift
  run "u_$name" 120 rocprofv3 --pmc "$@" -d "$O/u_$name" -o u_$name --output-format csv -- ./tools/ubench_quads o
done
if [ -z "$NO_BENCH" ]; then
  run b_kt 300 rocprofv3 --kernel-trace --stats -d "$O/b_kt" -o b_kt --output-format csv -- python3 $B
  for p in "${P[@]}"; do
    set -- $p; name=$1; shift
    run "b_$name" 300 rocprofv3 --pmc "$@" -d "$O/b_$name" -o b_$name --output-format csv -- python3 $B
  done
fi
find "$O" -name "*counter_collection.csv" | head -20
