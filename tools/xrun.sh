# A/B timing of experimental builds: rocprofv3 kernel stats of a short bench per library.
#   [BENCH_ARGS=...] [TAG=x] bash tools/xrun.sh lib1.so lib2.so ...   (paths relative to lego-loam-bor_amd/lego_amd)
TAG=${TAG:-x}
mkdir -p gpurun_out/$TAG
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for l in "$@"; do
  LEGO_FRONTEND_LIB=lego-loam-bor_amd/lego_amd/$l timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/$TAG/$l -o run -- python3 bench.py --no-cpu-baseline --steps 5 --warmup 2 $BENCH_ARGS > gpurun_out/$TAG/$l.log 2>&1 || exit 1
done
