# Heap-pop rewrite check: sort parity tests, the recorded-ring sort bench, bench lines (order 0 default).
set -e
TAG=$1
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python3 -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "sort or voxel or order" > "$OUT/tests.log" 2>&1
tail -2 "$OUT/tests.log"
LEGO_FRONTEND_LIB=lego-loam-bor_amd/lego_amd/liblego_frontend_prof.so timeout -k 10 120 python3 tools/sort_bench.py > "$OUT/sort_bench.txt" 2>&1
grep -v amdgpu.ids "$OUT/sort_bench.txt"
for i in 1 2; do
  timeout -k 10 300 python3 bench.py --no-cpu-baseline --roofline-streams 0 > "$OUT/bench$i.log" 2>&1
  echo "[$i] $(grep -o '"value": [0-9.]*' "$OUT/bench$i.log" | head -1) alt $(grep -o '"other_voxel_tie_order": {[^}]*}' "$OUT/bench$i.log")"
done
echo done
