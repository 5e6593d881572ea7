# Round-6 measurement set, from the repo root through gpurun:   tools/r06_final.sh TAG tests|bench|pmc|sweep|c5|latency
#   tests:   the whole -m gpu suite (LEGO_REPORT_DIR: the drift report) + smoke
#   bench:   the default bench line (C3 order 0 + order 1 beside it, C5, the S = 2048 pair, CPU baselines), a kernel
#            trace + stats of the measured pass split by bench pass, the C4 line
#   pmc:     FETCH_SIZE / WRITE_SIZE passes: C3 at S = 256 on the shipped layout, the S = 2048 roofline pair, C4
#   sweep:   C3 at S = 256 / 512 / 1024, both VoxelGrid orders (one line each)
#   c5:      C5's per-rank workloads on one GPU (80 / 40 / 20 / 10 sequences: rank 0 of N = 1 / 2 / 4 / 8)
#   latency: config C2's mode, one scan in flight through the single-context C-ABI, both orders, two repeats
set -e
TAG=$1; WHAT=$2
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
if [ "$WHAT" = tests ]; then
  LEGO_REPORT_DIR=$OUT timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > "$OUT/gpu_tests.log" 2>&1
  tail -3 "$OUT/gpu_tests.log"
  timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > "$OUT/smoke.log" 2>&1
  tail -2 "$OUT/smoke.log"
fi
if [ "$WHAT" = bench ]; then
  timeout -k 10 400 python3 bench.py --steps 20 --warmup 5 > "$OUT/bench.log" 2>&1
  tail -c 300 "$OUT/bench.log"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/stats" -o run -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-alt-order --roofline-streams 0 --no-c5 > "$OUT/bench_traced.log" 2>&1
  find "$OUT/stats" -name '*kernel_trace.csv' -exec cp {} "$OUT/kernel_trace.csv" \;
  find "$OUT/stats" -name '*kernel_stats.csv' -exec cp {} "$OUT/kernel_stats.csv" \;
  python3 tools/trace_split.py "$OUT/kernel_trace.csv" "$OUT/kernel_trace_split.csv" --steps 20 --warmup 5 > "$OUT/split.txt"
  python3 tools/timeline.py "$OUT/kernel_trace.csv" --steps 20 --warmup 5 > "$OUT/timeline.txt"
  tail -n 1 "$OUT/split.txt"
  timeout -k 10 400 python3 bench.py --kind hdl64 --steps 20 --warmup 5 --no-cpu-baseline --no-c5 > "$OUT/bench_hdl64.log" 2>&1
  tail -c 300 "$OUT/bench_hdl64.log"
fi
if [ "$WHAT" = pmc ]; then
  P="--steps 4 --warmup 2 --no-cpu-baseline --no-alt-order --roofline-streams 0 --no-c5"
  timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/fetch" -o run -- python3 bench.py $P > "$OUT/fetch.log" 2>&1
  timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/write" -o run -- python3 bench.py $P > "$OUT/write.log" 2>&1
  timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/fetch2048" -o run -- python3 tools/roofline_pmc.py 2048 > "$OUT/fetch2048.log" 2>&1
  timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/write2048" -o run -- python3 tools/roofline_pmc.py 2048 > "$OUT/write2048.log" 2>&1
  timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/fetch_hdl" -o run -- python3 bench.py --kind hdl64 $P > "$OUT/fetch_hdl.log" 2>&1
  timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/write_hdl" -o run -- python3 bench.py --kind hdl64 $P > "$OUT/write_hdl.log" 2>&1
  python3 tools/pmc_summarize.py "$OUT/fetch" "$OUT/write" "$OUT/pmc.json" --workload vlp16 --streams 256
  python3 tools/pmc_summarize.py "$OUT/fetch2048" "$OUT/write2048" "$OUT/pmc_2048.json" --workload vlp16 --streams 2048
  python3 tools/pmc_summarize.py "$OUT/fetch_hdl" "$OUT/write_hdl" "$OUT/hdl64_pmc.json" --workload hdl64 --streams 256
fi
if [ "$WHAT" = sweep ]; then
  for S in 256 512 1024; do
    for O in 0 1; do
      timeout -k 10 300 python3 bench.py --streams $S --steps 20 --warmup 5 --no-cpu-baseline --no-alt-order --roofline-streams 0 --no-c5 --voxel-tie-order $O > "$OUT/sweep_s${S}_o${O}.log" 2>&1
      tail -n 1 "$OUT/sweep_s${S}_o${O}.log" >> "$OUT/streams_sweep.jsonl"
      echo "S=$S order $O: $(grep -o '"value": [0-9.]*' "$OUT/sweep_s${S}_o${O}.log" | head -1)"
    done
  done
fi
if [ "$WHAT" = c5 ]; then
  for NSEQ in 80 40 20 10; do
    timeout -k 10 300 python3 bench.py --config c5 --c5-sequences $NSEQ --no-cpu-baseline --no-alt-order --roofline-streams 0 > "$OUT/c5_$NSEQ.log" 2>&1
    grep '^{' "$OUT/c5_$NSEQ.log" | tail -1 >> "$OUT/c5_per_rank.jsonl"
    echo "c5 $NSEQ: $(grep -o '"value": [0-9.]*' "$OUT/c5_$NSEQ.log" | head -1)"
  done
fi
if [ "$WHAT" = latency ]; then
  for rep in 1 2; do
    for O in 0 1; do
      timeout -k 10 200 python3 tools/latency.py --voxel-order $O >> "$OUT/latency_one_scan.jsonl" 2>/dev/null
    done
  done
  cat "$OUT/latency_one_scan.jsonl"
fi
echo done
