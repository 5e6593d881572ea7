# A/B over environment settings of the working tree: sort check, sort bench, then one bench line per setting
mkdir -p gpurun_out/env
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 250 --timeout-method thread > gpurun_out/env/tests.log 2>&1
rc=$?; tail -2 gpurun_out/env/tests.log; [ $rc -eq 0 ] || exit $rc
if [ -n "$TEST_ENV" ]; then
  env $TEST_ENV timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 250 --timeout-method thread > gpurun_out/env/tests2.log 2>&1
  rc=$?; tail -2 gpurun_out/env/tests2.log; [ $rc -eq 0 ] || exit $rc
fi
LEGO_FRONTEND_LIB=lego-loam-bor_amd/lego_amd/liblego_frontend_prof.so timeout -k 10 120 python tools/sort_bench.py > gpurun_out/env/sort_bench.log 2>&1
rc=$?; grep total gpurun_out/env/sort_bench.log; [ $rc -eq 0 ] || exit $rc
i=0
for e in "$@"; do
  i=$((i+1))
  env $e timeout -k 10 200 python bench.py --no-cpu-baseline --roofline-streams 0 > gpurun_out/env/bench_$i.log 2>&1 || exit 1
  echo "[$e] $(grep -o '"value": [0-9.]*' gpurun_out/env/bench_$i.log | head -1) $(grep -o '"other_voxel_tie_order": {[^}]*}' gpurun_out/env/bench_$i.log) $(grep -o '"stages_ms": {[^}]*}' gpurun_out/env/bench_$i.log)"
done
