# Round-4 (second session) quick GPU check: selected GPU tests, then bench lines at the given lags.
#   tools/r04b_check.sh TAG "pytest -k expression" "lag list" [bench args...]
set -e
TAG=$1; KEXPR=$2; LAGS=$3; shift 3
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
if [ -n "$KEXPR" ]; then
  timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "$KEXPR" > "$OUT/tests.log" 2>&1
  tail -3 "$OUT/tests.log"
fi
for L in $LAGS; do
  timeout -k 10 300 python3 bench.py --lag $L --no-cpu-baseline --roofline-streams 0 "$@" > "$OUT/bench_lag$L.log" 2>&1
  tail -n 1 "$OUT/bench_lag$L.log" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('lag $L', d['value'], d['ms_per_step'], d.get('other_voxel_tie_order'))"
done
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$OUT/trace" -o run -- python3 bench.py --no-cpu-baseline --roofline-streams 0 --no-alt-order --lag ${LAGS##* } "$@" > "$OUT/bench_traced.log" 2>&1
find "$OUT/trace" -name '*kernel_trace.csv' -exec cp {} "$OUT/kernel_trace.csv" \;
echo done
