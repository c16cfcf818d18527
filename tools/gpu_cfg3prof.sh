#!/bin/bash
# configs[2]: phase stamps of k_scan_chunks (diagnostic build) and rocprofv3 kernel stats of tools/bench_configs.py cfg3.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out
export TMPDIR=/tmp
CASK_LIB_PATH=cask_amd/build/stamps/libcask_scan.so timeout -k 10 200 python -u tools/stamps.py --zipf-gib 4 > gpurun_out/stz.log 2>&1
rc=$?; echo "stamps rc=$rc"; grep -v amdgpu.ids gpurun_out/stz.log | tail -14; [ $rc -ne 0 ] && exit $rc
rm -rf gpurun_out/prof_cfg3
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_cfg3 -o kt --output-format csv -- python3 tools/bench_configs.py cfg3 --out gpurun_out/cfg3_prof.json > gpurun_out/prof_cfg3.log 2>&1
rc=$?; echo "prof rc=$rc"; find gpurun_out/prof_cfg3 -name "*stats*.csv"
exit $rc
