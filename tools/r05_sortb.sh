set -e
OUT=gpurun_out/$1
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
LEGO_FRONTEND_LIB=lego-loam-bor_amd/lego_amd/liblego_frontend_prof.so timeout -k 10 120 python3 tools/sort_bench.py > "$OUT/sort_bench.txt" 2>&1
cat "$OUT/sort_bench.txt"
