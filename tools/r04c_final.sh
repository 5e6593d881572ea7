# Round-4 final measurement set (second session), from the repo root through gpurun:
#   tools/r04c_final.sh TAG tests|bench|pmc
#   tests: the whole -m gpu suite; bench: the default bench line, a kernel trace + stats of the
#   measured pass (tools/trace_split.py), the HDL-64E line and the streams sweep;
#   pmc: FETCH_SIZE / WRITE_SIZE passes (C3 at S = 256 and the S = 2048 roofline pair, C4).
set -e
TAG=$1; WHAT=$2
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
if [ "$WHAT" = tests ]; then
  timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > "$OUT/gpu_tests.log" 2>&1
  tail -3 "$OUT/gpu_tests.log"
  timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > "$OUT/smoke.log" 2>&1
  tail -2 "$OUT/smoke.log"
fi
if [ "$WHAT" = bench ]; then
  timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 > "$OUT/bench.log" 2>&1
  tail -c 300 "$OUT/bench.log"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/stats" -o run -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-alt-order > "$OUT/bench_traced.log" 2>&1
  find "$OUT/stats" -name '*kernel_trace.csv' -exec cp {} "$OUT/kernel_trace.csv" \;
  find "$OUT/stats" -name '*kernel_stats.csv' -exec cp {} "$OUT/kernel_stats.csv" \;
  timeout -k 10 300 python3 bench.py --kind hdl64 --steps 20 --warmup 5 --no-cpu-baseline > "$OUT/bench_hdl64.log" 2>&1
  tail -c 300 "$OUT/bench_hdl64.log"
  for S in 256 512 1024; do
    for O in 0 1; do
      timeout -k 10 200 python3 bench.py --streams $S --voxel-tie-order $O --steps 20 --no-cpu-baseline --no-alt-order --roofline-streams 0 > "$OUT/sweep_s${S}_o${O}.log" 2>&1
      tail -n 1 "$OUT/sweep_s${S}_o${O}.log" >> "$OUT/streams_sweep.jsonl"
    done
  done
fi
if [ "$WHAT" = pmc ]; then
  timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/fetch" -o run -- python3 bench.py --steps 4 --warmup 2 --no-cpu-baseline --no-alt-order --roofline-streams 0 > "$OUT/fetch.log" 2>&1
  timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/write" -o run -- python3 bench.py --steps 4 --warmup 2 --no-cpu-baseline --no-alt-order --roofline-streams 0 > "$OUT/write.log" 2>&1
  timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/fetch2048" -o run -- python3 tools/roofline_pmc.py 2048 > "$OUT/fetch2048.log" 2>&1
  timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/write2048" -o run -- python3 tools/roofline_pmc.py 2048 > "$OUT/write2048.log" 2>&1
  timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/fetch_hdl" -o run -- python3 bench.py --kind hdl64 --steps 4 --warmup 2 --no-cpu-baseline --no-alt-order --roofline-streams 0 > "$OUT/fetch_hdl.log" 2>&1
  timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/write_hdl" -o run -- python3 bench.py --kind hdl64 --steps 4 --warmup 2 --no-cpu-baseline --no-alt-order --roofline-streams 0 > "$OUT/write_hdl.log" 2>&1
  timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/fetch_hdl2048" -o run -- python3 tools/roofline_pmc.py 2048 hdl64 > "$OUT/fetch_hdl2048.log" 2>&1
  timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/write_hdl2048" -o run -- python3 tools/roofline_pmc.py 2048 hdl64 > "$OUT/write_hdl2048.log" 2>&1
fi
echo done
