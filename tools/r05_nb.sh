# k_pw_scatter batches a workgroup (VLP-16, S >= 64): roofline pair and throughput per build.
set -e
TAG=$1
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
C="--steps 20 --warmup 5 --no-cpu-baseline --no-alt-order --roofline-streams 0 --no-c5 --voxel-tie-order 0"
for rep in 1 2; do
  for L in liblego_frontend.so liblego_frontend_nb2.so liblego_frontend_nb1.so; do
    LEGO_FRONTEND_LIB=lego-loam-bor_amd/lego_amd/$L timeout -k 10 200 python3 bench.py $C > "$OUT/s.log" 2>&1
    echo "$L: $(grep -o '"value": [0-9.]*' "$OUT/s.log" | head -1) $(grep -o '"frac": [0-9.]*' "$OUT/s.log" | head -1) $(grep -o '"per_kernel": {[^}]*}[^}]*}' "$OUT/s.log")" | tee -a "$OUT/nb.txt"
  done
done
