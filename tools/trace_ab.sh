# kernel traces of the default bench for the working tree and the variants staged under ab_tmp/, then the
# HDL-64E (C4) PMC passes (FETCH_SIZE and WRITE_SIZE in separate runs)
set -e
mkdir -p gpurun_out/tr
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
R=$GRAFT_REPO_ROOT
for rev in ${REVS:-cur}; do
  if [ "$rev" = "cur" ]; then d=$R; else d=$R/ab_tmp/$rev; fi
  (cd $d && timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/tr/$rev -o run -- python3 bench.py --no-cpu-baseline --roofline-streams 0 ${BENCH_ARGS} > $R/gpurun_out/tr/bench_$rev.log 2>&1)
  echo "$rev: $(grep -o '"value": [0-9.]*' gpurun_out/tr/bench_$rev.log | head -1)"
done
if [ -n "$HDL" ]; then
  timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/tr/hdl_fetch -o run -- python3 bench.py --kind hdl64 --steps 4 --warmup 2 --no-cpu-baseline --no-alt-order --roofline-streams 0 > gpurun_out/tr/hdl_fetch.log 2>&1
  timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/tr/hdl_write -o run -- python3 bench.py --kind hdl64 --steps 4 --warmup 2 --no-cpu-baseline --no-alt-order --roofline-streams 0 > gpurun_out/tr/hdl_write.log 2>&1
  echo hdl pmc done
fi
