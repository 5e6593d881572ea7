# round-3 GPU check: parity tests, then the voxel probe (phase timers + order-0 kernel trace)
mkdir -p gpurun_out
export LEGO_REPORT_DIR=gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread ${TEST_ARGS} > gpurun_out/gpu_tests.log 2>&1
rc=$?
tail -3 gpurun_out/gpu_tests.log
[ $rc -eq 0 ] || exit $rc
bash tools/voxel_probe.sh r03v
