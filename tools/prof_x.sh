mkdir -p gpurun_out/px
LEGO_FRONTEND_LIB=lego-loam-bor_amd/lego_amd/liblego_frontend_prof.so timeout -k 10 200 python3 tools/phase_profile.py 256 1 > gpurun_out/px/phase1.log 2>&1
grep -E "^x|segments|rings|ring " gpurun_out/px/phase1.log
