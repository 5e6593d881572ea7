# Schedule / layout A/B of bench.py variants on one box (round 5):  tools/r05_ab.sh TAG
set -e
TAG=$1
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
C="--steps 20 --warmup 5 --no-cpu-baseline --no-alt-order --roofline-streams 0 --no-c5"
for rep in 1 2; do
  for v in "0 -1 2" "0 0 1" "0 0 2" "0 1 1" "1 0 1" "1 1 2"; do
    set -- $v
    timeout -k 10 200 python3 bench.py $C --voxel-tie-order $1 --wide $2 --lag $3 > "$OUT/ab.log" 2>&1
    echo "order $1 wide $2 lag $3: $(grep -o '"value": [0-9.]*' "$OUT/ab.log" | head -1) $(grep -o '"stages_ms": {[^}]*}' "$OUT/ab.log")" | tee -a "$OUT/ab.txt"
  done
done
echo done
