mkdir -p gpurun_out
bash tools/_gpu_check.sh && \
LEGO_FRONTEND_LIB=lego-loam-bor_amd/lego_amd/liblego_frontend_exp.so timeout -k 10 200 python bench.py --no-cpu-baseline --no-alt-order > gpurun_out/bench_exp.log 2>&1
grep metric gpurun_out/bench_exp.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('EXP', d['value'], d['stages_ms'])"
