# One iteration of the VoxelGrid work (round 5): sort tests, the recorded-ring sort bench, both orders' bench
# lines with the VoxelGrid alone.   tools/r05_iter.sh TAG
set -e
TAG=$1
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "sort or noise_free or vlp16_sequence or bench_schedule" > "$OUT/tests.log" 2>&1
tail -2 "$OUT/tests.log"
LEGO_FRONTEND_LIB=lego-loam-bor_amd/lego_amd/liblego_frontend_prof.so timeout -k 10 120 python3 tools/sort_bench.py > "$OUT/sort_bench.txt" 2>&1
grep "c10 \|c110" "$OUT/sort_bench.txt"
C="--steps 20 --warmup 5 --no-cpu-baseline --no-alt-order --roofline-streams 0 --no-c5"
for O in 0 1; do
  timeout -k 10 200 python3 bench.py $C --voxel-tie-order $O > "$OUT/b$O.log" 2>&1
  echo "order $O: $(grep -o '"value": [0-9.]*' "$OUT/b$O.log" | head -1) $(grep -o '"stages_ms": {[^}]*}' "$OUT/b$O.log")"
done
echo done
