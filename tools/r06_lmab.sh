# Round 6: few-stream LM A/B (tools/few_streams.py over library variants) after a parity subset.
#   TAG=... LIBS="..." TESTS="..." bash tools/r06_lmab.sh
set -e
OUT=gpurun_out/${TAG:-r06q}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
if [ -n "$TESTS" ]; then
  timeout -k 10 700 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "$TESTS" > "$OUT/tests.log" 2>&1 || { tail -30 "$OUT/tests.log"; exit 1; }
  tail -n 2 "$OUT/tests.log"
fi
for L in ${LIBS:-liblego_frontend.so}; do
  for a in ${CASES:-"10 60 0" "20 60 0" "40 60 0" "80 60 0" "10 60 1"}; do
    echo "$L $(LEGO_FRONTEND_LIB=lego-loam-bor_amd/lego_amd/$L timeout -k 10 120 python3 tools/few_streams.py $a 2>&1 | grep -v amdgpu.ids)" | tee -a $OUT/few.txt
  done
done
