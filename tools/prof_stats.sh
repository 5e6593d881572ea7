# rocprofv3 kernel trace + stats of the default bench command (run through gpurun from the repo root)
TAG=${1:-cur}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/stats" -o run -- python3 bench.py --no-cpu-baseline > "$OUT/bench_traced.log" 2>&1
