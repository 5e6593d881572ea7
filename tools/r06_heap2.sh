# Two-pops-in-flight heap sort (round 6): sort + VoxelGrid parity tests on the new build, the recorded-ring
# (round 6: also the two-pops-in-flight variant, tools/ab/r06_heap_pipeline.patch, built as liblego_frontend{,_prof}.so beside the shipped _base builds)
# sort bench on both profile builds, then C3 bench lines of both builds (A/B).   tools/r06_heap2.sh TAG
set -e
TAG=$1
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "sort or noise_free or vlp16_sequence or voxel or map or bench_schedule" > "$OUT/tests.log" 2>&1 || { tail -40 "$OUT/tests.log"; exit 1; }
tail -2 "$OUT/tests.log"
for P in base_prof prof; do
  LEGO_FRONTEND_LIB=lego-loam-bor_amd/lego_amd/liblego_frontend_$P.so timeout -k 10 120 python3 tools/sort_bench.py > "$OUT/sort_bench_$P.txt" 2>&1
  echo "== $P"; grep -v amdgpu.ids "$OUT/sort_bench_$P.txt"
done
LIBS="liblego_frontend_base.so liblego_frontend.so liblego_frontend_base.so liblego_frontend.so" bash tools/r06_quick.sh $TAG none
