# k_voxel probe: phase timers (profile build) for both VoxelGrid tie orders, then a kernel trace of the
# order-0 bench (run through gpurun from the repo root)
TAG=${1:-r03v}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
LEGO_FRONTEND_LIB=lego-loam-bor_amd/lego_amd/liblego_frontend_prof.so timeout -k 10 240 python tools/phase_profile.py 256 0 > "$OUT/phase0.txt" 2>&1 && \
LEGO_FRONTEND_LIB=lego-loam-bor_amd/lego_amd/liblego_frontend_prof.so timeout -k 10 240 python tools/phase_profile.py 256 1 > "$OUT/phase1.txt" 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/stats" -o run -- python3 bench.py --no-cpu-baseline --voxel-tie-order 0 --no-alt-order --roofline-streams 0 > "$OUT/bench0.log" 2>&1
