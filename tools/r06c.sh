# Round 6: projection-only A/B of library variants (tools/proj_time.py); LIBS / TESTS override.
set -e
OUT=gpurun_out/${TAG:-r06c}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
if [ -n "$TESTS" ]; then
  timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "$TESTS" > "$OUT/tests.log" 2>&1 || { tail -30 "$OUT/tests.log"; exit 1; }
  tail -n 1 "$OUT/tests.log"
fi
for L in ${LIBS:-liblego_frontend.so liblego_frontend_tp.so}; do
  for K in vlp16 hdl64; do
    LEGO_FRONTEND_LIB=lego-loam-bor_amd/lego_amd/$L timeout -k 10 120 python3 tools/proj_time.py $K 256 1 >> $OUT/proj_time.txt 2>&1
  done
done
cat $OUT/proj_time.txt
if [ -n "$PMC" ]; then
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY --output-format csv -d $OUT/sq -o run -- python3 tools/proj_time.py vlp16 256 1 > $OUT/sq.log 2>&1
echo pmc-done
fi
if [ -n "$TRACE" ]; then
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt -o run -- python3 tools/proj_time.py ${TRACE} 256 1 > $OUT/kt.log 2>&1
find $OUT/kt -name '*kernel_stats.csv' -exec cp {} $OUT/kernel_stats.csv \;
python3 - $OUT/kernel_stats.csv <<'PY'
import csv, sys
for r in csv.reader(open(sys.argv[1])):
    if r[0] == 'Name' or 'pw_' in r[0] or 'fa_prep' in r[0]: print(r[0][:60], r[1:4])
PY
fi
