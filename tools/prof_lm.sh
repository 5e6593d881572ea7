# LM phase profile (profile build) + GPU check
mkdir -p gpurun_out/plm
LEGO_FRONTEND_LIB=lego-loam-bor_amd/lego_amd/liblego_frontend_prof.so timeout -k 10 200 python3 tools/phase_profile.py 256 1 > gpurun_out/plm/phase1.log 2>&1
grep -E "^lm" gpurun_out/plm/phase1.log
