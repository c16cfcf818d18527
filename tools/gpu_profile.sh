#!/bin/bash
# One GPU call: full bench line, rocprofv3 kernel-trace stats, and two PMC passes (FETCH_SIZE,
# WRITE_SIZE) for the HBM traffic of the headline's dominant kernel (bench.py: configs[2]). Outputs under gpurun_out/; tools/pmc_summary.py
# turns them into profiles/.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out
TAG=${TAG:-r01}
step() {
  local name=$1 to=$2; shift 2
  echo "=== $name"; date
  timeout -k 10 "$to" "$@" > "$R/gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "rc=$rc"; tail -${TAILN:-3} "$R/gpurun_out/$name.log"
  if [ $rc -ne 0 ]; then echo "STOP after $name (rc=$rc)"; exit $rc; fi
}
if [ -z "$SKIP_BENCH" ]; then
  TAILN=1 step bench_full 600 python bench.py
fi
export TMPDIR=/tmp
B="$R/bench.py --steps ${PSTEPS:-20} --warmup ${PWARM:-3} --no-cpu-baseline --no-e2e --no-cfg1 --no-shard-n1 --no-cold"
rm -rf "$R/gpurun_out/prof_$TAG"
TAILN=1 step prof_kt 600 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_$TAG/kt" -o kt --output-format csv -- python3 $B
step prof_fetch 600 rocprofv3 --pmc FETCH_SIZE -d "$R/gpurun_out/prof_$TAG/fetch" -o fetch --output-format csv -- python3 $B
step prof_write 600 rocprofv3 --pmc WRITE_SIZE -d "$R/gpurun_out/prof_$TAG/write" -o write --output-format csv -- python3 $B
# memory-side read requests by size: FETCH_SIZE x2 under-reports nontemporal whole-line reads (round 5:
# 31.5 GB for k_run_hash's 34.4 GB of log bytes), the request count does not
step prof_rdreq 600 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_128B_sum -d "$R/gpurun_out/prof_$TAG/rdreq" -o rdreq --output-format csv -- python3 $B
if [ -n "$CFG2" ]; then  # configs[2] (32 GiB Zipf): the same three passes over tools/bench_configs.py cfg3
  C="$R/tools/bench_configs.py cfg3 --steps 2"
  rm -rf "$R/gpurun_out/prof_${TAG}_cfg2"
  TAILN=1 step cfg2_kt 600 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_${TAG}_cfg2/kt" -o kt --output-format csv -- python3 $C
  step cfg2_fetch 600 rocprofv3 --pmc FETCH_SIZE -d "$R/gpurun_out/prof_${TAG}_cfg2/fetch" -o fetch --output-format csv -- python3 $C
  step cfg2_write 600 rocprofv3 --pmc WRITE_SIZE -d "$R/gpurun_out/prof_${TAG}_cfg2/write" -o write --output-format csv -- python3 $C
fi
find "$R/gpurun_out/prof_$TAG"* -name "*.csv" | head -20
