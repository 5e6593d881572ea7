# Round 6: C5's per-rank workloads on one GPU (SURVEY §8(e) model, not a scaling measurement).
# With contiguous sequence shards and no data-path collective, rank 0 of an N-GPU C5 run processes
# exactly `bench.py --config c5 --c5-sequences 80/N`.   tools/r06_c5rank.sh TAG [LIB]
set -e
TAG=$1
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
[ -n "$2" ] && export LEGO_FRONTEND_LIB=lego-loam-bor_amd/lego_amd/$2
for NSEQ in 80 40 20 10; do
  timeout -k 10 300 python3 bench.py --config c5 --c5-sequences $NSEQ --no-cpu-baseline > "$OUT/c5_$NSEQ.log" 2>&1
  grep '^{' "$OUT/c5_$NSEQ.log" | tail -1 >> "$OUT/c5_per_rank.jsonl"
  echo "c5 $NSEQ: $(grep -o '"value": [0-9.]*' "$OUT/c5_$NSEQ.log" | head -1)"
done
C="--steps 20 --warmup 5 --no-cpu-baseline --no-alt-order --roofline-streams 0 --no-c5"
timeout -k 10 200 python3 bench.py $C > "$OUT/b0.log" 2>&1
echo "c3 order 0: $(grep -o '"value": [0-9.]*' "$OUT/b0.log" | head -1)"
echo done
