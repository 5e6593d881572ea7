# Order-0 VoxelGrid A/B on the GPU: the recorded-ring sort bench (profile build) for both emulations, then
# kernel traces (with --stats) of the default bench with the level-synchronous sort and with the stack one.
#   tools/r04_sortab.sh TAG
set -e
TAG=$1
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
LEGO_FRONTEND_LIB=lego-loam-bor_amd/lego_amd/liblego_frontend_prof.so timeout -k 10 120 python3 tools/sort_bench.py > "$OUT/sort_bench.txt" 2>&1
cat "$OUT/sort_bench.txt"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/stack" -o run -- python3 bench.py --no-cpu-baseline --roofline-streams 0 --no-alt-order > "$OUT/bench_stack.log" 2>&1
tail -c 300 "$OUT/bench_stack.log"
LEGO_VOXEL_SORT=level timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/level" -o run -- python3 bench.py --no-cpu-baseline --roofline-streams 0 --no-alt-order > "$OUT/bench_level.log" 2>&1
tail -c 300 "$OUT/bench_level.log"
echo done
