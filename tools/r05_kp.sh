# C3 order 0: wide 1 vs wide 2 (one-workgroup k_project + wide segmentation), default and capped k_project.
set -e
TAG=$1
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
C="--steps 20 --warmup 5 --no-cpu-baseline --no-alt-order --roofline-streams 0 --no-c5 --voxel-tie-order 0"
for rep in 1 2; do
  for V in "liblego_frontend.so --wide 1" "liblego_frontend.so --wide 2" "liblego_frontend_kp96.so --wide 2" "liblego_frontend_kp96.so --wide 0"; do
    set -- $V
    LEGO_FRONTEND_LIB=lego-loam-bor_amd/lego_amd/$1 timeout -k 10 200 python3 bench.py $C $2 $3 > "$OUT/s.log" 2>&1
    echo "$V: $(grep -o '"value": [0-9.]*' "$OUT/s.log" | head -1) $(grep -o '"frac": [0-9.]*' "$OUT/s.log" | head -1) $(grep -o '"project": [0-9.]*' "$OUT/s.log")" | tee -a "$OUT/kp.txt"
  done
done
