set -e
LIBS="liblego_frontend.so liblego_frontend_u4.so liblego_frontend_lx.so liblego_frontend_tp.so" ORDERS=0 HDL=1 bash tools/r06_quick.sh r06b "input_orders or hdl64_parity"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r06b/stats -o run -- python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-alt-order --roofline-streams 0 --no-c5 > gpurun_out/r06b/traced.log 2>&1
find gpurun_out/r06b/stats -name '*kernel_stats.csv' -exec cp {} gpurun_out/r06b/kernel_stats.csv \;
echo traced
