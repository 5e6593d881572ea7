# Layout / lag A/B for C3 order 0 on one box (round 5):  tools/r05_sched2.sh TAG
set -e
TAG=$1
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
C="--steps 20 --warmup 5 --no-cpu-baseline --no-alt-order --roofline-streams 0 --no-c5 --voxel-tie-order 0"
for rep in 1 2; do
  for A in "--wide 0 --lag 1" "--wide 1 --lag 1" "--wide 1 --lag 2" "--wide 0 --lag 2" "--wide 2 --lag 1"; do
    timeout -k 10 200 python3 bench.py $C $A > "$OUT/s.log" 2>&1
    echo "$A: $(grep -o '"value": [0-9.]*' "$OUT/s.log" | head -1) $(grep -o '"lm": [0-9.]*' "$OUT/s.log")" | tee -a "$OUT/sched.txt"
  done
done
