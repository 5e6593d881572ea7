# LM iteration (round 5): LM-related parity tests, the per-scan k_lm log (profile build), bench lines.
set -e
TAG=$1
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "vlp16_sequence or hdl64 or injected or kdtree or tie or bench_schedule or batch" > "$OUT/tests.log" 2>&1 || { tail -40 "$OUT/tests.log"; exit 1; }
tail -2 "$OUT/tests.log"
LEGO_FRONTEND_LIB=lego-loam-bor_amd/lego_amd/liblego_frontend_prof.so timeout -k 10 200 python3 tools/lm_log.py 256 1 > "$OUT/lmlog_o1.txt" 2>&1; head -3 "$OUT/lmlog_o1.txt"
LEGO_FRONTEND_LIB=lego-loam-bor_amd/lego_amd/liblego_frontend_prof.so timeout -k 10 300 python3 tools/lm_log.py 256 1 hdl64 > "$OUT/lmlog_hdl_o1.txt" 2>&1; head -3 "$OUT/lmlog_hdl_o1.txt"
HDL=${HDL:-1} bash tools/r05_quick.sh $TAG none
