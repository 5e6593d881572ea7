# Quick GPU iteration (round 5): a -k subset of the GPU tests, then bench lines of both VoxelGrid orders
# (C3) and, with HDL=1, of C4.   tools/r05_quick.sh TAG "pytest -k expression"
set -e
TAG=$1
K=${2:-"sort or noise_free or vlp16_sequence or bench_schedule"}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
if [ "$K" != none ]; then
  timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "$K" > "$OUT/tests.log" 2>&1
  tail -2 "$OUT/tests.log"
fi
C="--steps 20 --warmup 5 --no-cpu-baseline --no-alt-order --roofline-streams 0 --no-c5"
for O in 0 1; do
  timeout -k 10 200 python3 bench.py $C --voxel-tie-order $O > "$OUT/b$O.log" 2>&1
  echo "order $O: $(grep -o '"value": [0-9.]*' "$OUT/b$O.log" | head -1) $(grep -o '"stages_ms": {[^}]*}' "$OUT/b$O.log")"
done
if [ "${HDL:-0}" = 1 ]; then
  for O in 0 1; do
    timeout -k 10 300 python3 bench.py --kind hdl64 $C --voxel-tie-order $O > "$OUT/h$O.log" 2>&1
    echo "hdl64 order $O: $(grep -o '"value": [0-9.]*' "$OUT/h$O.log" | head -1) $(grep -o '"stages_ms": {[^}]*}' "$OUT/h$O.log")"
  done
fi
echo done
