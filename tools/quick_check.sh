# quick GPU check: selected parity tests, then the default bench (both VoxelGrid orders) -> gpurun_out/
mkdir -p gpurun_out
export LEGO_REPORT_DIR=gpurun_out
timeout -k 10 400 python -u -m pytest ${TESTS:-tests/test_gpu_parity.py} -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/quick_tests.log 2>&1
rc=$?
tail -3 gpurun_out/quick_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --no-cpu-baseline --roofline-streams 0 ${BENCH_ARGS} > gpurun_out/quick_bench.log 2>&1
rc=$?
tail -c 600 gpurun_out/quick_bench.log
exit $rc
