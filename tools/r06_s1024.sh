# Round 6: the stable VoxelGrid order at 512 / 1,024 streams under each layout and lag, and a kernel trace
# of the default schedule at 1,024.   tools/r06_s1024.sh TAG
set -e
OUT=gpurun_out/$1
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
C="--steps 20 --warmup 5 --no-cpu-baseline --no-alt-order --roofline-streams 0 --no-c5 --voxel-tie-order 1"
for S in 512 1024; do
  for W in -1 0 1; do
    for G in "" "--lag 2"; do
      timeout -k 10 300 python3 bench.py $C --streams $S --wide $W $G > "$OUT/s${S}_w${W}_$G.log" 2>&1 || true
      echo "S=$S wide=$W $G: $(grep -o '"value": [0-9.]*' "$OUT/s${S}_w${W}_$G.log" | head -1) $(grep -o '"stages_ms": {[^}]*}' "$OUT/s${S}_w${W}_$G.log")" | tee -a $OUT/sched.txt
    done
  done
done
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/kt -o run -- python3 bench.py $C --streams 1024 > $OUT/kt.log 2>&1
find $OUT/kt -name '*kernel_trace.csv' -exec cp {} $OUT/kernel_trace.csv \;
python3 tools/timeline.py $OUT/kernel_trace.csv --steps 20 --warmup 5 > $OUT/timeline.txt
head -60 $OUT/timeline.txt
