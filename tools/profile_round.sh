#!/bin/bash
# Round profile on the GPU box (run through gpurun from the repo root):
#   bash tools/profile_round.sh r01
# 1. rocprofv3 kernel trace + stats of the default bench command;
# 2. two separate PMC passes (FETCH_SIZE, WRITE_SIZE; MI355X_MICROARCH.md: they do not fit one pass);
# 3. the plain bench line (VLP-16, C3), the reference-exact VoxelGrid order and the HDL-64E-like config (C4).
# Afterwards, here: tools/trace_split.py and tools/pmc_summarize.py write profiles/<tag>_*.
set -e
TAG=${1:-r01}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/stats" -o run -- python3 bench.py --no-cpu-baseline > "$OUT/bench_traced.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/fetch" -o run -- python3 bench.py --steps 4 --warmup 2 --no-cpu-baseline > "$OUT/fetch.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/write" -o run -- python3 bench.py --steps 4 --warmup 2 --no-cpu-baseline > "$OUT/write.log" 2>&1
timeout -k 10 300 python3 bench.py > "$OUT/bench.log" 2>&1
timeout -k 10 300 python3 bench.py --voxel-tie-order 0 --no-cpu-baseline > "$OUT/bench_order0.log" 2>&1
timeout -k 10 300 python3 bench.py --kind hdl64 --no-cpu-baseline > "$OUT/bench_hdl64.log" 2>&1
