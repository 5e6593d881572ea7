# A/B: parity tests of the working tree, then the default bench of each revision staged under ab_tmp/
mkdir -p gpurun_out/ab
export LEGO_REPORT_DIR=gpurun_out
timeout -k 10 400 python -u -m pytest ${TESTS:-tests/test_gpu_parity.py} -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/ab/tests.log 2>&1
rc=$?
tail -3 gpurun_out/ab/tests.log
[ $rc -eq 0 ] || exit $rc
for rev in ${REVS}; do
  if [ "$rev" = "cur" ]; then d=.; else d=ab_tmp/$rev; fi
  (cd $d && timeout -k 10 200 python bench.py --no-cpu-baseline --roofline-streams 0 > $GRAFT_REPO_ROOT/gpurun_out/ab/bench_$rev.log 2>&1) || exit 1
  echo "$rev: $(grep -o '"value": [0-9.]*' gpurun_out/ab/bench_$rev.log | head -1) $(grep -o '"other_voxel_tie_order": {[^}]*}' gpurun_out/ab/bench_$rev.log)"
done
if [ -n "$PROBE" ]; then
  cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/ab/probe_fetch -o run -- python3 tools/fetch_probe.py > gpurun_out/ab/probe.log 2>&1 || exit 1
  timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/ab/probe_write -o run -- python3 tools/fetch_probe.py >> gpurun_out/ab/probe.log 2>&1 || exit 1
  echo probe done
fi
