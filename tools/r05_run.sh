# Round-5 measurement set, from the repo root through gpurun:
#   tools/r05_run.sh TAG tests|bench|trace|pmc|hdl|sweep [more modes...]
#   tests: the whole -m gpu suite (LEGO_REPORT_DIR=gpurun_out/TAG: the drift report) + smoke
#   bench: the default bench line (C3 headline, order 1 beside it, C5, roofline at 2048, CPU baseline)
#   trace: rocprofv3 kernel trace + stats of the measured pass only (--no-alt-order --roofline-streams 0
#          --no-c5), split by bench pass (tools/trace_split.py)
#   pmc:   FETCH_SIZE / WRITE_SIZE passes of the same command (C3), then of C4
#   hdl:   the C4 (HDL-64E) bench line
#   sweep: streams sweep 256 / 512 / 1024 for both VoxelGrid orders
set -e
TAG=$1; shift
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
B="--steps 20 --warmup 5"
for WHAT in "$@"; do
  echo "== $WHAT"
  if [ "$WHAT" = tests ]; then
    LEGO_REPORT_DIR=$OUT timeout -k 10 1100 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > "$OUT/gpu_tests.log" 2>&1
    tail -3 "$OUT/gpu_tests.log"
    timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > "$OUT/smoke.log" 2>&1
    tail -2 "$OUT/smoke.log"
  fi
  if [ "$WHAT" = quick ]; then
    LEGO_REPORT_DIR=$OUT timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "$QUICK_K" > "$OUT/gpu_quick.log" 2>&1
    tail -3 "$OUT/gpu_quick.log"
  fi
  if [ "$WHAT" = bench ]; then
    timeout -k 10 400 python3 bench.py $B > "$OUT/bench.log" 2>&1
    tail -c 600 "$OUT/bench.log"
  fi
  if [ "$WHAT" = trace ]; then
    timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/stats" -o run -- python3 bench.py $B --no-cpu-baseline --no-alt-order --roofline-streams 0 --no-c5 > "$OUT/bench_traced.log" 2>&1
    find "$OUT/stats" -name '*kernel_trace.csv' -exec cp {} "$OUT/kernel_trace.csv" \;
    find "$OUT/stats" -name '*kernel_stats.csv' -exec cp {} "$OUT/kernel_stats.csv" \;
    python3 tools/trace_split.py "$OUT/kernel_trace.csv" "$OUT/kernel_trace_split.csv" --steps 20 --warmup 5 > "$OUT/split.txt"
    tail -n 2 "$OUT/split.txt"
    tail -c 300 "$OUT/bench_traced.log"
  fi
  if [ "$WHAT" = pmc ]; then
    timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/fetch" -o run -- python3 bench.py --steps 4 --warmup 2 --no-cpu-baseline --no-alt-order --roofline-streams 0 --no-c5 > "$OUT/fetch.log" 2>&1
    timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/write" -o run -- python3 bench.py --steps 4 --warmup 2 --no-cpu-baseline --no-alt-order --roofline-streams 0 --no-c5 > "$OUT/write.log" 2>&1
    timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/fetch_hdl" -o run -- python3 bench.py --kind hdl64 --steps 4 --warmup 2 --no-cpu-baseline --no-alt-order --roofline-streams 0 --no-c5 > "$OUT/fetch_hdl.log" 2>&1
    timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/write_hdl" -o run -- python3 bench.py --kind hdl64 --steps 4 --warmup 2 --no-cpu-baseline --no-alt-order --roofline-streams 0 --no-c5 > "$OUT/write_hdl.log" 2>&1
    echo pmc done
  fi
  if [ "$WHAT" = phase ]; then
    for O in 0 1; do
      LEGO_FRONTEND_LIB=lego-loam-bor_amd/lego_amd/liblego_frontend_prof.so timeout -k 10 300 python3 tools/phase_profile.py 256 $O > "$OUT/phase_order$O.txt" 2>&1
      grep "voxel\|sort:" "$OUT/phase_order$O.txt" | head -8
    done
  fi
  if [ "$WHAT" = hdl ]; then
    timeout -k 10 400 python3 bench.py --kind hdl64 $B --no-cpu-baseline --no-c5 > "$OUT/bench_hdl64.log" 2>&1
    tail -c 400 "$OUT/bench_hdl64.log"
  fi
  if [ "$WHAT" = sweep ]; then
    for S in 256 512 1024; do
      for O in 0 1; do
        timeout -k 10 200 python3 bench.py --streams $S --voxel-tie-order $O --steps 20 --no-cpu-baseline --no-alt-order --roofline-streams 0 --no-c5 > "$OUT/sweep_s${S}_o${O}.log" 2>&1
        tail -n 1 "$OUT/sweep_s${S}_o${O}.log" >> "$OUT/streams_sweep.jsonl"
      done
    done
    echo sweep done
  fi
done
echo done
