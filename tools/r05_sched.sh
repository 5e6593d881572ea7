# Schedule A/B on one box (round 5): C3 order 0 / 1 at lag 1 and lag 2, twice.   tools/r05_sched.sh TAG
set -e
TAG=$1
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
C="--steps 20 --warmup 5 --no-cpu-baseline --no-alt-order --roofline-streams 0 --no-c5"
for rep in 1 2; do
  for A in "--voxel-tie-order 0 --lag 1" "--voxel-tie-order 0 --lag 2" "--voxel-tie-order 1 --lag 1" "--voxel-tie-order 1 --lag 2" $EXTRA; do
    timeout -k 10 200 python3 bench.py $C $A > "$OUT/s.log" 2>&1
    echo "$A: $(grep -o '"value": [0-9.]*' "$OUT/s.log" | head -1) $(grep -o '"lm": [0-9.]*' "$OUT/s.log")" | tee -a "$OUT/sched.txt"
  done
done
