# A/B timing of experimental builds: rocprofv3 kernel stats of a short bench per library.
#   bash tools/xrun.sh lib1.so lib2.so ...   (paths relative to lego-loam-bor_amd/lego_amd)
mkdir -p gpurun_out/x
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for l in "$@"; do
  LEGO_FRONTEND_LIB=lego-loam-bor_amd/lego_amd/$l timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/x/$l -o run -- python3 bench.py --no-cpu-baseline --steps 5 --warmup 2 > gpurun_out/x/$l.log 2>&1 || exit 1
done
