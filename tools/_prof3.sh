mkdir -p gpurun_out/p3
bash tools/_gpu_check.sh && \
LEGO_FRONTEND_LIB=lego-loam-bor_amd/lego_amd/liblego_frontend_prof.so timeout -k 10 120 python3 tools/sort_bench.py > gpurun_out/p3/sort.log 2>&1 && \
LEGO_FRONTEND_LIB=lego-loam-bor_amd/lego_amd/liblego_frontend_prof.so timeout -k 10 200 python3 tools/phase_profile.py 256 0 > gpurun_out/p3/phase0.log 2>&1
cat gpurun_out/p3/sort.log
