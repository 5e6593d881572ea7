# Round 6 A/B: parity subset on the default library, then bench lines (C3 both orders, C4) and C5 per-rank
# (10 / 80 sequences) for each library in LIBS, REPS times interleaved.   TAG=... LIBS="..." bash tools/r06_ab2.sh
set -e
OUT=gpurun_out/${TAG:-r06s}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
if [ -n "$TESTS" ]; then
  timeout -k 10 800 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "$TESTS" > "$OUT/tests.log" 2>&1 || { tail -30 "$OUT/tests.log"; exit 1; }
  tail -n 2 "$OUT/tests.log"
fi
C="--steps 20 --warmup 5 --no-cpu-baseline --no-alt-order --roofline-streams 0 --no-c5"
val() { grep -o '"value": [0-9.]*' "$1" | head -1 | cut -d' ' -f2; }
lm() { grep -o '"lm": [0-9.]*' "$1" | head -1 | cut -d' ' -f2; }
for rep in $(seq 1 ${REPS:-1}); do
for L in ${LIBS:-liblego_frontend.so}; do
  export LEGO_FRONTEND_LIB=lego-loam-bor_amd/lego_amd/$L
  timeout -k 10 200 python3 bench.py $C --voxel-tie-order 0 > "$OUT/b0_$L.log" 2>&1
  timeout -k 10 200 python3 bench.py $C --voxel-tie-order 1 > "$OUT/b1_$L.log" 2>&1
  timeout -k 10 300 python3 bench.py --kind hdl64 $C > "$OUT/h0_$L.log" 2>&1
  timeout -k 10 300 python3 bench.py --config c5 --c5-sequences 10 --no-cpu-baseline --no-alt-order --roofline-streams 0 > "$OUT/c10_$L.log" 2>&1
  timeout -k 10 300 python3 bench.py --config c5 --c5-sequences 80 --no-cpu-baseline --no-alt-order --roofline-streams 0 > "$OUT/c80_$L.log" 2>&1
  echo "$L rep $rep: C3o0 $(val $OUT/b0_$L.log) (lm $(lm $OUT/b0_$L.log))  C3o1 $(val $OUT/b1_$L.log) (lm $(lm $OUT/b1_$L.log))  C4 $(val $OUT/h0_$L.log) (lm $(lm $OUT/h0_$L.log))  C5/10 $(val $OUT/c10_$L.log)  C5/80 $(val $OUT/c80_$L.log)" | tee -a $OUT/ab.txt
done
done
