# Per-scan k_lm log (profile build): C3 both orders, C4 order 1.   tools/r05_lmlog.sh TAG
set -e
TAG=$1
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export LEGO_FRONTEND_LIB=lego-loam-bor_amd/lego_amd/liblego_frontend_prof.so
timeout -k 10 200 python3 tools/lm_log.py 256 1 > "$OUT/lmlog_o1.txt" 2>&1; cat "$OUT/lmlog_o1.txt"
timeout -k 10 200 python3 tools/lm_log.py 256 0 > "$OUT/lmlog_o0.txt" 2>&1; cat "$OUT/lmlog_o0.txt"
timeout -k 10 300 python3 tools/lm_log.py 256 1 hdl64 > "$OUT/lmlog_hdl_o1.txt" 2>&1; cat "$OUT/lmlog_hdl_o1.txt"
