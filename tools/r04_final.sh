# Round-4 measurement set (through gpurun from the repo root), after the test suite:
#  1. the default bench line (C3, voxel_tie_order 0, the other order beside it); 2. kernel trace + stats of
#  it (split by pass: tools/trace_split.py); 3. C3 PMC passes (FETCH_SIZE / WRITE_SIZE separately);
#  4. the S = 2048 roofline pair's PMC passes; 5. C4 (HDL-64E) bench; 6. C4 PMC passes.
#   tools/r04_final.sh TAG [skip-pmc]
set -e
TAG=${1:-r04}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python3 bench.py > "$OUT/bench.log" 2>&1
tail -c 400 "$OUT/bench.log"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/stats" -o run -- python3 bench.py --no-cpu-baseline --no-alt-order > "$OUT/bench_traced.log" 2>&1
find "$OUT/stats" -name '*kernel_trace.csv' -exec cp {} "$OUT/kernel_trace.csv" \;
find "$OUT/stats" -name '*kernel_stats.csv' -exec cp {} "$OUT/kernel_stats.csv" \;
timeout -k 10 300 python3 bench.py --kind hdl64 --no-cpu-baseline > "$OUT/bench_hdl64.log" 2>&1
tail -c 300 "$OUT/bench_hdl64.log"
if [ "$2" != "skip-pmc" ]; then
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/fetch" -o run -- python3 bench.py --steps 4 --warmup 2 --no-cpu-baseline --no-alt-order --roofline-streams 0 > "$OUT/fetch.log" 2>&1
timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/write" -o run -- python3 bench.py --steps 4 --warmup 2 --no-cpu-baseline --no-alt-order --roofline-streams 0 > "$OUT/write.log" 2>&1
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/fetch2048" -o run -- python3 tools/roofline_pmc.py 2048 > "$OUT/fetch2048.log" 2>&1
timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/write2048" -o run -- python3 tools/roofline_pmc.py 2048 > "$OUT/write2048.log" 2>&1
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/fetch_hdl" -o run -- python3 bench.py --kind hdl64 --steps 4 --warmup 2 --no-cpu-baseline --no-alt-order --roofline-streams 0 > "$OUT/fetch_hdl.log" 2>&1
timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/write_hdl" -o run -- python3 bench.py --kind hdl64 --steps 4 --warmup 2 --no-cpu-baseline --no-alt-order --roofline-streams 0 > "$OUT/write_hdl.log" 2>&1
fi
echo done
