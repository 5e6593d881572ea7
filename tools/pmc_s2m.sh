# SQ issue / wait breakdown and L2 hit rate of k_s2m (two rocprofv3 --pmc passes over a short
# tools/bench_s2m.py run), from the repo root through gpurun:  bash tools/pmc_s2m.sh TAG
TAG=${1:-s2mpmc}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -s KILL 180 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_WAVES --kernel-include-regex k_s2m --output-format csv -d "$OUT/sq" -o run -- python3 tools/bench_s2m.py --streams 256 --reps 2 --warmup 1 --cpu-sample 1 > "$OUT/sq.log" 2>&1 &&
timeout -s KILL 180 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --kernel-include-regex k_s2m --output-format csv -d "$OUT/tcc" -o run -- python3 tools/bench_s2m.py --streams 256 --reps 2 --warmup 1 --cpu-sample 1 > "$OUT/tcc.log" 2>&1
