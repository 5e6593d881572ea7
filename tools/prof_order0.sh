mkdir -p gpurun_out/prof0
export LEGO_FRONTEND_LIB=lego-loam-bor_amd/lego_amd/liblego_frontend_prof.so
timeout -k 10 200 python tools/phase_profile.py 256 0 > gpurun_out/prof0/phase_o0.txt 2>&1 && \
timeout -k 10 200 python tools/phase_profile.py 256 1 > gpurun_out/prof0/phase_o1.txt 2>&1 && \
unset LEGO_FRONTEND_LIB && cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof0/stats -o run -- python3 bench.py --no-cpu-baseline --voxel-tie-order 0 > gpurun_out/prof0/bench_traced.log 2>&1
