# Round-4 (second session) baseline: default bench line, then a kernel trace (with stats) of the
# measured order-0 pass for timeline analysis (tools/timeline.py).
#   tools/r04b_base.sh TAG [bench args...]
set -e
TAG=$1; shift
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python3 bench.py --no-cpu-baseline --roofline-streams 0 "$@" > "$OUT/bench.log" 2>&1
tail -c 600 "$OUT/bench.log"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- python3 bench.py --no-cpu-baseline --roofline-streams 0 --no-alt-order "$@" > "$OUT/bench_traced.log" 2>&1
find "$OUT/trace" -name '*kernel_trace.csv' -exec cp {} "$OUT/kernel_trace.csv" \;
find "$OUT/trace" -name '*kernel_stats.csv' -exec cp {} "$OUT/kernel_stats.csv" \;
echo done
