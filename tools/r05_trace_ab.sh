# Kernel traces of the throughput pass for two library builds (round 5):  tools/r05_trace_ab.sh TAG LIB_B [BENCH_ARGS]
set -e
TAG=$1; LIBB=$2; shift 2
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
C="--steps 20 --warmup 5 --no-cpu-baseline --no-alt-order --roofline-streams 0 --no-c5"
for lib in liblego_frontend.so $LIBB; do
  LEGO_FRONTEND_LIB=lego-loam-bor_amd/lego_amd/$lib timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$OUT/t_$lib" -o run -- python3 bench.py $C "$@" > "$OUT/t_$lib.log" 2>&1
  find "$OUT/t_$lib" -name '*kernel_trace.csv' -exec cp {} "$OUT/trace_$lib.csv" \;
  python3 tools/timeline.py "$OUT/trace_$lib.csv" --steps 20 --warmup 5 > "$OUT/timeline_$lib.txt"
  echo "$lib: $(grep -o '"value": [0-9.]*' "$OUT/t_$lib.log" | head -1)"
done
