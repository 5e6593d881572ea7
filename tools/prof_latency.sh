# Kernel + memory-copy trace of the one-scan-in-flight latency run (run through gpurun from the repo root)
TAG=${1:-lat}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 120 python3 tools/latency.py --scans 40 > "$OUT/latency.log" 2>&1 && \
timeout -k 10 200 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv -d "$OUT/trace" -o run -- python3 tools/latency.py --scans 40 > "$OUT/latency_traced.log" 2>&1
