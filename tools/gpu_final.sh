#!/bin/bash
# Round-end evidence in one call: parity suite, full bench line, configs[2] + compaction
# measurements, rocprofv3 kernel stats of configs[2], then the headline profile (kernel stats +
# FETCH_SIZE / WRITE_SIZE passes, tools/gpu_profile.sh).
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out
export TMPDIR=/tmp
bash tools/gpu_tests.sh || exit $?
timeout -k 10 500 python -u tools/bench_configs.py cfg3 compact --out gpurun_out/configs_final.json > gpurun_out/configs_final.log 2>&1
rc=$?; echo "configs rc=$rc"; tail -c 1500 gpurun_out/configs_final.log; [ $rc -ne 0 ] && exit $rc
rm -rf gpurun_out/prof_cfg3
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_cfg3 -o kt --output-format csv -- python3 tools/bench_configs.py cfg3 --out gpurun_out/cfg3_prof.json > gpurun_out/prof_cfg3.log 2>&1
rc=$?; echo "prof cfg3 rc=$rc"; [ $rc -ne 0 ] && exit $rc
TAG=${TAG:-r01e} bash tools/gpu_profile.sh
