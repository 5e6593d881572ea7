# Per-ring VoxelGrid timing (profile build): C3 order 0 / 1, C4 order 0.   tools/r05_ringlog.sh TAG
set -e
TAG=$1
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export LEGO_FRONTEND_LIB=lego-loam-bor_amd/lego_amd/liblego_frontend_prof.so
timeout -k 10 200 python3 tools/ring_log.py 256 0 > "$OUT/ringlog_o0.txt" 2>&1; cat "$OUT/ringlog_o0.txt"
timeout -k 10 200 python3 tools/ring_log.py 256 1 > "$OUT/ringlog_o1.txt" 2>&1; cat "$OUT/ringlog_o1.txt"
timeout -k 10 300 python3 tools/ring_log.py 256 0 hdl64 > "$OUT/ringlog_hdl_o0.txt" 2>&1; cat "$OUT/ringlog_hdl_o0.txt"
