# sort check + sort bench (both algorithms), then traces / HDL PMC (tools/trace_ab.sh)
mkdir -p gpurun_out/tr
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "sort_matches" -m gpu -x -q --timeout 250 --timeout-method thread > gpurun_out/tr/sort_test.log 2>&1
rc=$?; tail -2 gpurun_out/tr/sort_test.log; [ $rc -eq 0 ] || exit $rc
LEGO_FRONTEND_LIB=lego-loam-bor_amd/lego_amd/liblego_frontend_prof.so timeout -k 10 120 python tools/sort_bench.py > gpurun_out/tr/sort_bench.log 2>&1
rc=$?; cat gpurun_out/tr/sort_bench.log | grep -v amdgpu.ids; [ $rc -eq 0 ] || exit $rc
bash tools/trace_ab.sh
