set -e
mkdir -p gpurun_out/p1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/p1/m0 -o run -- python3 bench.py --no-cpu-baseline --no-alt-order --voxel-tie-order 0 > gpurun_out/p1/m0.log 2>&1
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/p1/m1 -o run -- python3 bench.py --no-cpu-baseline --no-alt-order --voxel-tie-order 1 > gpurun_out/p1/m1.log 2>&1
LEGO_FRONTEND_LIB=lego-loam-bor_amd/lego_amd/liblego_frontend_prof.so timeout -k 10 200 python3 tools/phase_profile.py 256 0 > gpurun_out/p1/phase0.log 2>&1
LEGO_FRONTEND_LIB=lego-loam-bor_amd/lego_amd/liblego_frontend_prof.so timeout -k 10 200 python3 tools/phase_profile.py 256 1 > gpurun_out/p1/phase1.log 2>&1
