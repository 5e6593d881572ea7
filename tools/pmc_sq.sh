# SQ issue / wait breakdown per kernel (one rocprofv3 --pmc pass, <= 8 SQ counters), run through
# gpurun from the repo root:  bash tools/pmc_sq.sh TAG
TAG=${1:-sq}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_WAVES --output-format csv -d "$OUT/pmc" -o run -- python3 bench.py --steps 4 --warmup 2 --no-cpu-baseline > "$OUT/run.log" 2>&1
