# A/B of library builds: parity tests on the default library (TESTS=..., SKIP_TESTS=1 to skip), then the
# default bench per library (LIBS="liblego_frontend.so liblego_frontend_x.so", relative to lego_amd/).
mkdir -p gpurun_out/ab
export LEGO_REPORT_DIR=gpurun_out
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 500 python -u -m pytest ${TESTS:-tests/test_gpu_parity.py} -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/ab/tests.log 2>&1
  rc=$?
  tail -3 gpurun_out/ab/tests.log
  [ $rc -eq 0 ] || { grep -E 'Error|assert|FAILED' gpurun_out/ab/tests.log | head -20; exit $rc; }
fi
for rep in 1 ${REPS:+$(seq 2 $REPS)}; do
for l in ${LIBS:-liblego_frontend.so}; do
  LEGO_FRONTEND_LIB=lego-loam-bor_amd/lego_amd/$l timeout -k 10 200 python bench.py --no-cpu-baseline --roofline-streams ${RS:-0} ${BENCH_ARGS:---no-alt-order} > gpurun_out/ab/bench_${l}_$rep.log 2>&1 || { tail -20 gpurun_out/ab/bench_${l}_$rep.log; exit 1; }
  python3 - "$l" gpurun_out/ab/bench_${l}_$rep.log <<'PY'
import json, sys
line = [l for l in open(sys.argv[2]) if l.startswith('{')][-1]
d = json.loads(line)
r = d["roofline"]
print(sys.argv[1], "value %.1f" % d["value"], "frac %.4f" % r["frac"], "pair_ms %.4f" % r["launch_ms"],
      {k: v["ms"] for k, v in r["per_kernel"].items()}, "stages", d.get("stages_ms"),
      "alt", (d.get("other_voxel_tie_order") or {}).get("value"))
PY
done
done
