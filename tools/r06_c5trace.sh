# Round 6: few-stream (C5 per-rank) probes + a kernel trace of the 10-stream run.   tools/r06_c5trace.sh TAG
set -e
OUT=gpurun_out/$1
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for a in "10 60 0 auto" "10 60 0 1" "10 60 0 0" "10 60 1 auto" "20 60 0 auto" "40 60 0 auto"; do
  timeout -k 10 120 python3 tools/few_streams.py $a 2>&1 | grep -v amdgpu.ids | tee -a $OUT/few.txt
done
timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d $OUT/kt -o run -- python3 tools/few_streams.py 10 60 0 > $OUT/kt.log 2>&1
find $OUT/kt -name '*kernel_trace.csv' -exec cp {} $OUT/kernel_trace.csv \;
python3 tools/timeline.py $OUT/kernel_trace.csv --steps 8 --warmup 40 > $OUT/timeline.txt
tail -n 60 $OUT/timeline.txt
