# Round-4 quick GPU check: selected parity tests, then bench lines (order 0 with the stack emulation of
# the VoxelGrid sort, the level-synchronous sort for A/B, and order 1).
#   tools/r04_check.sh TAG "pytest -k expression"
set -e
TAG=$1; KEXPR=$2
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
if [ -n "$KEXPR" ]; then
  timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "$KEXPR" > "$OUT/tests.log" 2>&1
  tail -3 "$OUT/tests.log"
fi
timeout -k 10 300 python3 bench.py --voxel-tie-order 0 --no-cpu-baseline --roofline-streams 0 > "$OUT/bench0.log" 2>&1
tail -c 600 "$OUT/bench0.log"
LEGO_VOXEL_SORT=level timeout -k 10 300 python3 bench.py --voxel-tie-order 0 --no-cpu-baseline --roofline-streams 0 --no-alt-order > "$OUT/bench0_level.log" 2>&1
tail -c 300 "$OUT/bench0_level.log"
echo done
