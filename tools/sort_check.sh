# device sort parity + sort bench variants + default bench (both tie orders)
mkdir -p gpurun_out/srt
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 250 --timeout-method thread > gpurun_out/srt/tests.log 2>&1
rc=$?; tail -2 gpurun_out/srt/tests.log; [ $rc -eq 0 ] || exit $rc
LEGO_FRONTEND_LIB=lego-loam-bor_amd/lego_amd/liblego_frontend_prof.so timeout -k 10 200 python tools/sort_bench.py > gpurun_out/srt/sort_bench.log 2>&1
rc=$?; grep total gpurun_out/srt/sort_bench.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python bench.py --no-cpu-baseline --roofline-streams 0 > gpurun_out/srt/bench.log 2>&1 || exit 1
echo "$(grep -o '"value": [0-9.]*' gpurun_out/srt/bench.log | head -1) $(grep -o '"other_voxel_tie_order": {[^}]*}' gpurun_out/srt/bench.log)"
