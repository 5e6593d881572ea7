# A/B of several library builds on one box (round 5):  LIBS="a.so b.so ..." tools/r05_abn.sh TAG BENCH_ARGS...
# (libraries relative to lego-loam-bor_amd/lego_amd/; the first is usually the shipped one)
set -e
TAG=$1; shift
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
C="--steps 20 --warmup 5 --no-cpu-baseline --no-alt-order --roofline-streams 0 --no-c5"
for rep in $(seq 1 ${REPS:-2}); do
  for lib in $LIBS; do
    LEGO_FRONTEND_LIB=lego-loam-bor_amd/lego_amd/$lib timeout -k 10 200 python3 bench.py $C "$@" > "$OUT/ab.log" 2>&1
    echo "$lib $*: $(grep -o '"value": [0-9.]*' "$OUT/ab.log" | head -1) $(grep -o '"stages_ms": {[^}]*}' "$OUT/ab.log")" | tee -a "$OUT/ab.txt"
  done
done
