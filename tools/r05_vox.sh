# VoxelGrid cost probe (round 5): the recorded-ring sort bench (profile build) and the VoxelGrid stage alone
# (bench.py stages_ms.voxel_alone) for both tie orders.   tools/r05_vox.sh TAG
set -e
TAG=$1
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
LEGO_FRONTEND_LIB=lego-loam-bor_amd/lego_amd/liblego_frontend_prof.so timeout -k 10 120 python3 tools/sort_bench.py > "$OUT/sort_bench.txt" 2>&1
cat "$OUT/sort_bench.txt"
C="--steps 20 --warmup 5 --no-cpu-baseline --no-alt-order --roofline-streams 0 --no-c5"
for O in 0 1; do
  timeout -k 10 200 python3 bench.py $C --voxel-tie-order $O > "$OUT/b$O.log" 2>&1
  echo "order $O: $(grep -o '"value": [0-9.]*' "$OUT/b$O.log" | head -1) $(grep -o '"stages_ms": {[^}]*}' "$OUT/b$O.log")"
done
echo done
