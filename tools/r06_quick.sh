# Quick GPU iteration (round 6): a -k subset of the GPU tests, then bench lines (C3 order 0, order 1;
# HDL=1 adds C4 order 0) with the roofline pair.   tools/r06_quick.sh TAG "pytest -k expression" [LIBS]
set -e
TAG=$1
K=${2:-"wide or input_orders or hdl64 or bench_schedule or edge or hbm_stage"}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
if [ "$K" != none ]; then
  timeout -k 10 700 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "$K" > "$OUT/tests.log" 2>&1 || { tail -30 "$OUT/tests.log"; exit 1; }
  tail -2 "$OUT/tests.log"
fi
C="--steps 20 --warmup 5 --no-cpu-baseline --no-alt-order --roofline-streams 0 --no-c5"
summ() {
python3 - "$1" <<'PY'
import json, sys
line = [l for l in open(sys.argv[1]) if l.startswith('{')][-1]
d = json.loads(line); r = d["roofline"]
print("value %.1f" % d["value"], "frac %.4f" % r["frac"], "pair_ms %.4f" % r["launch_ms"],
      {k: v["ms"] for k, v in r.get("per_kernel", {}).items()}, "stages", d.get("stages_ms"))
PY
}
for L in ${LIBS:-liblego_frontend.so}; do
  export LEGO_FRONTEND_LIB=lego-loam-bor_amd/lego_amd/$L
  for O in ${ORDERS:-0 1}; do
    timeout -k 10 200 python3 bench.py $C --voxel-tie-order $O > "$OUT/b${O}_$L.log" 2>&1
    echo "$L order $O: $(summ "$OUT/b${O}_$L.log")"
  done
  if [ "${HDL:-0}" = 1 ]; then
    timeout -k 10 300 python3 bench.py --kind hdl64 $C > "$OUT/h0_$L.log" 2>&1
    echo "$L hdl64 order 0: $(summ "$OUT/h0_$L.log")"
  fi
done
echo done
