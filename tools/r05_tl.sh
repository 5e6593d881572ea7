# Full GPU suite + smoke, then a kernel trace (timeline, split by pass) of the default order-0 bench.   tools/r05_tl.sh TAG
set -e
TAG=$1
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
LEGO_REPORT_DIR=$OUT timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$OUT/gpu_tests.log" 2>&1 || { tail -30 "$OUT/gpu_tests.log"; exit 1; }
tail -2 "$OUT/gpu_tests.log"
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1
tail -1 "$OUT/smoke.log"
B="--steps 20 --warmup 5"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/stats" -o run -- python3 bench.py $B --no-cpu-baseline --no-alt-order --roofline-streams 0 --no-c5 > "$OUT/bench_traced.log" 2>&1
find "$OUT/stats" -name '*kernel_trace.csv' -exec cp {} "$OUT/kernel_trace.csv" \;
find "$OUT/stats" -name '*kernel_stats.csv' -exec cp {} "$OUT/kernel_stats.csv" \;
python3 tools/trace_split.py "$OUT/kernel_trace.csv" "$OUT/kernel_trace_split.csv" --steps 20 --warmup 5 > "$OUT/split.txt"
python3 tools/timeline.py "$OUT/kernel_trace.csv" --steps 20 --warmup 5 > "$OUT/timeline.txt"
tail -n 3 "$OUT/split.txt"
grep -o '"value": [0-9.]*' "$OUT/bench_traced.log" | head -1
