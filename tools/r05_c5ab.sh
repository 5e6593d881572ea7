# C5 (80 sequences x 250 scans on one GPU): layout / lag A/B.   tools/r05_c5ab.sh TAG
set -e
OUT=gpurun_out/$1
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
C="--streams 8 --steps 2 --warmup 1 --no-cpu-baseline --no-alt-order --roofline-streams 0 --config c5"
for O in 0 1; do
  for v in "0 1" "0 2" "1 1" "1 2"; do
    set -- $v
    timeout -k 10 200 python3 bench.py $C --voxel-tie-order $O --wide $1 --lag $2 > "$OUT/c5.log" 2>&1
    echo "order $O wide $1 lag $2: c5 $(grep -o '"c5": {[^}]*}' "$OUT/c5.log" | grep -o '"value": [0-9.]*')" | tee -a "$OUT/c5ab.txt"
  done
done
