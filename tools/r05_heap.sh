# Heap-sort iteration (round 5): sort + VoxelGrid parity tests, the recorded-ring sort bench (profile build),
# the per-ring VoxelGrid log, then the C3 bench lines of both orders.   tools/r05_heap.sh TAG
set -e
TAG=$1
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "sort or noise_free or vlp16_sequence or voxel or map" > "$OUT/tests.log" 2>&1 || { tail -40 "$OUT/tests.log"; exit 1; }
tail -2 "$OUT/tests.log"
LEGO_FRONTEND_LIB=lego-loam-bor_amd/lego_amd/liblego_frontend_prof.so timeout -k 10 120 python3 tools/sort_bench.py > "$OUT/sort_bench.txt" 2>&1
cat "$OUT/sort_bench.txt"
LEGO_FRONTEND_LIB=lego-loam-bor_amd/lego_amd/liblego_frontend_prof.so timeout -k 10 200 python3 tools/ring_log.py 256 0 > "$OUT/ringlog_o0.txt" 2>&1
head -4 "$OUT/ringlog_o0.txt"
bash tools/r05_quick.sh $TAG none
