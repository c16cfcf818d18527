#!/bin/bash
cd ${GRAFT_REPO_ROOT:-$(pwd)}; mkdir -p gpurun_out
for L in 0.39 0.5 0.6 0.7; do echo "L=$L"; XX_LOAD=$L timeout -k 10 200 python -u tools/merge_bench.py 52000000 2>&1 | grep -E "tables|lists|records:" || exit 1; done > gpurun_out/r06h_loadsweep.log 2>&1
cat gpurun_out/r06h_loadsweep.log
