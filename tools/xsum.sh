# Summaries of an xrun.sh A/B: timing-pass durations of the named kernels and each bench line.
#   bash tools/xsum.sh TAG 'k_project|k_fa_prep' lib1.so lib2.so ...
TAG=$1; PAT=$2; shift 2
for l in "$@"; do
  echo "== $l"
  python3 tools/trace_split.py gpurun_out/$TAG/$l/run_kernel_trace.csv /tmp/xsum_$l.csv --steps 5 --warmup 2 > /dev/null
  grep -E "$PAT" /tmp/xsum_$l.csv | grep timing_pass | cut -c1-120
  grep -h metric gpurun_out/$TAG/$l.log | python3 -c "
import sys, json
for l in sys.stdin:
    d = json.loads(l); print('  value', d['value'], 'stages', d['stages_ms'], 'frac', d['roofline']['frac'])"
done
