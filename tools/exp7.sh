mkdir -p gpurun_out/exp7
timeout -k 10 200 python bench.py --kind hdl64 --streams 64 --no-cpu-baseline > gpurun_out/exp7/hdl64.log 2>&1 && \
timeout -k 10 200 python bench.py --kind hdl64 --streams 256 --no-cpu-baseline > gpurun_out/exp7/hdl256.log 2>&1
