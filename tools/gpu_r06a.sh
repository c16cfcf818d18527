cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_compaction.py tests/test_rccl_ranks_gpu.py tests/test_scan_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r06a_tests.log 2>&1
rc=$?; tail -5 gpurun_out/r06a_tests.log; echo "pytest rc=$rc"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/r06a_bench.log 2>&1; rc=$?; tail -c 3000 gpurun_out/r06a_bench.log; exit $rc
