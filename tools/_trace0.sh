mkdir -p gpurun_out/t0
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/t0 -o run -- python3 bench.py --no-cpu-baseline --no-alt-order --voxel-tie-order 0 --steps 6 --warmup 2 > gpurun_out/t0/bench.log 2>&1
ls gpurun_out/t0
