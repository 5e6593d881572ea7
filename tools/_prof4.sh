mkdir -p gpurun_out/p3
LEGO_FRONTEND_LIB=lego-loam-bor_amd/lego_amd/liblego_frontend_prof.so timeout -k 10 200 python3 tools/phase_profile.py 256 0 > gpurun_out/p3/phase0.log 2>&1
grep -E "^(x:voxel|  sort)" gpurun_out/p3/phase0.log
