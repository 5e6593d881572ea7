# quick GPU check: parity tests then the bench line (steps joined by &&)
mkdir -p gpurun_out
export LEGO_REPORT_DIR=gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread ${TEST_ARGS} > gpurun_out/gpu_tests.log 2>&1 && \
timeout -k 10 300 python bench.py --no-cpu-baseline ${BENCH_ARGS} > gpurun_out/bench.log 2>&1
rc=$?
tail -3 gpurun_out/gpu_tests.log
grep metric gpurun_out/bench.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['stages_ms'], d['roofline']['achieved'], d['roofline']['frac'], d.get('other_voxel_tie_order'), d['roofline'].get('at_roofline_streams'))"
exit $rc
